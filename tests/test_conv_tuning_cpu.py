"""Per-layer conv tuning (`ops.conv._pick`) under multi-rank agreement, on CPU with gloo.

The candidate timings are faked (no GPU here); what is tested is the control flow around them:
- a stream-K hand-off time-out seen by ONE rank makes EVERY rank raise and exclude the stream-K
  configs (no rank is left blocked in the next collective), and
- a candidate whose launch is refused by the checked launch (DAMD_LAUNCH -> RuntimeError
  "kernel launch failed") is dropped instead of aborting the tuning.
"""

import pytest

from tests.dist_utils import run_distributed


class _FakeExt:
    def conv_sk_cfg(self, c):
        return c == 15

    def conv_num_cfgs(self):
        return 20


def _patch(mp, rank, timeouts_on_rank):
    """mp: a pytest monkeypatch (in-process test) or None (a spawned worker, discarded afterwards)."""
    import determined_amd.ops as ops
    from determined_amd.ops import conv as C

    def setattr_(obj, name, value):
        if mp is not None:
            mp.setattr(obj, name, value)
        else:
            setattr(obj, name, value)

    setattr_(C, "_TUNE", {})
    setattr_(C, "_EXCLUDE", frozenset())
    setattr_(C, "_DB_LOADED", True)
    setattr_(C, "_TUNE_ON", True)
    setattr_(C, "_time_once", lambda fn, reps=3, rounds=2: fn())
    setattr_(C, "_time_quick", lambda fn: fn())
    setattr_(ops, "ext", lambda: _FakeExt())
    setattr_(ops, "conv_sk_timeouts", lambda device=None: 1 if rank == timeouts_on_rank else 0)
    setattr_(C.torch.cuda, "is_current_stream_capturing", lambda: False)
    return C


def _timeout_worker(rank, world):
    C = _patch(None, rank, timeouts_on_rank=1)
    cands = {3: lambda: 2.0 + rank, 15: lambda: 1.0}
    raised = False
    try:
        with C.agree_across_ranks():
            C._pick(("fwd", "shape"), cands, 3)
    except RuntimeError as e:
        raised = "timed out" in str(e)
    excluded = ("*", 15) in C._EXCLUDE
    # the next layer still tunes (and agrees) on every rank, without stream-K
    import determined_amd.ops as ops

    ops.conv_sk_timeouts = lambda device=None: 0
    with C.agree_across_ranks():
        nxt = C._pick(("fwd", "shape2"), {3: lambda: 2.0, 15: lambda: 1.0}, 3)
    return {"raised": raised, "excluded": excluded, "next": nxt}


def test_stream_k_timeout_on_one_rank_raises_on_every_rank():
    outs = run_distributed(_timeout_worker, world=2)
    for o in outs:
        assert o["raised"] and o["excluded"]
        assert o["next"] == 3  # stream-K config 15 is no longer a candidate


def _refused_worker(rank, world):
    C = _patch(None, rank, timeouts_on_rank=-1)

    def refused():
        raise RuntimeError("determined_amd kernel launch failed in damd_conv_fwd_launch (x:1): hipErrorInvalidValue")

    with C.agree_across_ranks():
        got = C._pick(("fwd", "s"), {0: refused, 1: lambda: 5.0 - rank, 2: lambda: 7.0}, 0)
    return got


def test_refused_launch_is_not_a_candidate():
    assert run_distributed(_refused_worker, world=2) == [1, 1]


def test_other_runtime_errors_propagate(monkeypatch):
    C = _patch(monkeypatch, 0, timeouts_on_rank=-1)

    def broken():
        raise RuntimeError("something else")

    with pytest.raises(RuntimeError, match="something else"):
        C._pick(("fwd", "x"), {0: broken, 1: lambda: 1.0}, 0)


def _prune_worker(rank, world):
    """7 candidates: the quick pass (agreed) keeps the near-best ones only, identically on every rank;
    rank 1's quick time of candidate 4 is noisy-fast but the mean keeps the ranks together."""
    C = _patch(None, rank, timeouts_on_rank=-1)
    full_timed = []
    quick = {0: 9.0, 1: 3.0, 2: 3.3, 3: 8.0, 4: 7.0 if rank == 0 else 1.0, 5: 3.6, 6: 20.0}
    C._time_quick = lambda fn: fn()[1]

    def full(fn, reps=3, rounds=2):
        c, _ = fn()
        full_timed.append(c)
        return {1: 3.1, 2: 2.9, 5: 3.0, 4: 1.0}[c]

    C._time_once = full
    cands = {c: (lambda c=c: (c, quick[c])) for c in quick}
    with C.agree_across_ranks():
        got = C._pick(("fwd", "p"), cands, 0)
    return {"got": got, "full": sorted(full_timed)}


def test_tuning_prunes_to_agreed_near_best_candidates():
    outs = run_distributed(_prune_worker, world=2)
    for o in outs:
        # agreed quick times: 1 -> 3.0, 2 -> 3.3, 5 -> 3.6, 4 -> 4.0 (> 1.25 x 3.0): 4 is pruned everywhere
        assert o["full"] == [1, 2, 5]
        assert o["got"] == 2
