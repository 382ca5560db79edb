"""Experimental APIs (reference: ``harness/determined/experimental``): the SDK ``client``,
unmanaged Core API v2 (``core_v2``)."""

from determined_amd.experimental import client
from determined_amd.experimental import core_v2
