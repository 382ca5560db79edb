"""determined_amd: an MI355X-native deep-learning training platform with Determined's capabilities.

Python API (mirrors ``determined``):
    from determined_amd import core, pytorch
    with core.init() as core_context: ...
    class MyTrial(pytorch.PyTorchTrial): ...

Compute path: PyTorch-ROCm + hand-written CDNA4 HIP kernels (``determined_amd.ops``) + RCCL over
xGMI (``determined_amd.parallel``).  Control plane: master / agent / CLI (``determined_amd.master``,
``determined_amd.agent``, ``determined_amd.cli``) with a native C++ searcher and scheduler.
"""

__version__ = "0.1.0"

from determined_amd._info import ClusterInfo, TrialInfo, get_cluster_info  # noqa: E402
from determined_amd.config import ExperimentConfig  # noqa: E402
from determined_amd.core import InvalidHP  # noqa: E402


def __getattr__(name):  # lazy heavy submodules
    import importlib

    if name in ("core", "pytorch", "ops", "parallel", "searcher", "storage", "models", "config", "experimental",
                "transformers", "tensorboard", "launch"):
        return importlib.import_module(f"determined_amd.{name}")
    raise AttributeError(name)
