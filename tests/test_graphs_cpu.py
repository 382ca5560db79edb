"""GraphedStep control flow on the CPU with a stand-in graph API: warm-up runs happen once, the step is
captured once and every call replays it, recapture() skips the warm-up (the GPU behaviour is covered by
tests/test_graphs_gpu.py)."""

import contextlib

import torch

from determined_amd.utils import graphs


class _FakeGraph:
    def __init__(self):
        self.replays = 0

    def replay(self):
        self.replays += 1


def test_graphed_step_warmup_capture_replay(monkeypatch):
    calls = {"eager": 0, "captured": 0}
    capturing = {"on": False}
    made = []

    class _Stream:
        def wait_stream(self, other):
            pass

    @contextlib.contextmanager
    def _graph(g, pool=None):
        capturing["on"] = True
        yield
        capturing["on"] = False

    def _new_graph():
        g = _FakeGraph()
        made.append(g)
        return g

    monkeypatch.setattr(torch.cuda, "Stream", _Stream)
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "current_stream", lambda: _Stream())
    monkeypatch.setattr(torch.cuda, "synchronize", lambda: None)
    monkeypatch.setattr(torch.cuda, "CUDAGraph", _new_graph)
    monkeypatch.setattr(torch.cuda, "graph", _graph)

    out = {"v": 0}

    def step():
        if capturing["on"]:
            calls["captured"] += 1
        else:
            calls["eager"] += 1
        out["v"] += 1
        return out

    g = graphs.GraphedStep(step, warmup=3)
    assert not g.captured
    results = [g() for _ in range(4)]
    r = results[-1]
    assert g.captured and calls["captured"] == 1 and calls["eager"] == 3
    assert len(made) == 1 and made[0].replays == 4 and r is out
    g.recapture()
    assert len(made) == 2 and calls["captured"] == 2
