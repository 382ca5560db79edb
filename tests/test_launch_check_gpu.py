"""Every HIP kernel launch is checked (csrc/common.h DAMD_LAUNCH): an invalid launch raises a Python
RuntimeError naming the launcher instead of leaving the output tensor unwritten."""

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext():
    import determined_amd.ops as ops

    return ops.ext()


def test_valid_launch_writes_output(ext):
    out = ext.debug_launch(1000, 0)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.ones_like(out))


@pytest.mark.parametrize("mode", [1, 2], ids=["lds_over_limit", "block_too_large"])
def test_invalid_launch_raises(ext, mode):
    with pytest.raises(RuntimeError, match="kernel launch failed in damd_debug_launch"):
        ext.debug_launch(1000, mode)
    # the error is consumed: the next valid launch works
    out = ext.debug_launch(64, 0)
    torch.cuda.synchronize()
    assert torch.equal(out, torch.ones_like(out))


def test_failed_launch_then_valid_launch_still_raises_for_the_failed_one(ext):
    """A failure is reported by the launch that failed, not masked by a later successful launch."""
    with pytest.raises(RuntimeError):
        ext.debug_launch(100, 2)
    assert torch.equal(ext.debug_launch(100, 0), torch.ones(100, device="cuda"))
