"""graphs.StaticGraph on the host (no GPU): garbage collection is OFF for exactly the duration of a capture and
restored afterwards, also when the captured function raises.  A collection during capture could run the
destructor of an older graph (or its memory pool) mid-capture, which HIP refuses from inside a destructor --
an abort, not an exception (the round-2 fix, commit 28f73b2)."""
import contextlib
import gc

import pytest
import torch

from multimodalemotionrecognition_amd import graphs as G


class _Stream:
    device = torch.device("cpu")

    def __init__(self, *a, **k):
        pass

    def wait_stream(self, other):
        pass


class _Graph:
    def replay(self):
        pass


@pytest.fixture
def fake_cuda(monkeypatch):
    seen = {}

    @contextlib.contextmanager
    def graph(g, stream=None):
        seen["capturing"] = True
        try:
            yield
        finally:
            seen["capturing"] = False

    monkeypatch.setattr(torch.cuda, "CUDAGraph", _Graph)
    monkeypatch.setattr(torch.cuda, "Stream", _Stream)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _Stream())
    monkeypatch.setattr(torch.cuda, "graph", graph)
    return seen


@pytest.mark.parametrize("initially", [True, False])
def test_gc_disabled_during_capture_only(fake_cuda, initially):
    (gc.enable if initially else gc.disable)()
    states = []
    try:
        def fn(x):
            states.append((gc.isenabled(), fake_cuda.get("capturing")))
            return x + 1

        g = G.StaticGraph(fn, [torch.zeros(3)])
        assert states == [(False, True)]
        assert gc.isenabled() is initially
        assert torch.equal(g.out, torch.ones(3))
    finally:
        gc.enable()


def test_gc_restored_when_capture_raises(fake_cuda):
    gc.enable()

    def bad(x):
        assert not gc.isenabled()
        raise RuntimeError("capture failed")

    with pytest.raises(RuntimeError):
        G.StaticGraph(bad, [torch.zeros(2)])
    assert gc.isenabled()
