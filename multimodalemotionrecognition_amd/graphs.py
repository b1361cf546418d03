"""HIP-graph capture of the fixed-shape launch schedules (the MI355X answer to a tracing compiler).

A train step issues ~360 kernel launches from Python; through ctypes each costs ~20 us of host time, so
the host, not the GPU, became the bound (tools/host_time.py).  The encoders' schedules are static for a
given input shape -- the frozen WavLM forward and the ResNet18 trunk forward/backward have no RNG and no
host decisions -- so each is captured once into a ``torch.cuda.CUDAGraph`` (hipGraph on ROCm: our ctypes
launches go to torch's current stream, which is the capture stream inside ``torch.cuda.graph``) and
replayed as ONE host call afterwards.  Inputs are copied into graph-owned static buffers; outputs are the
graph's static tensors.  A graph is keyed by its shapes and by the device addresses of every parameter
and buffer it reads, so moving / re-homing weights (``.to()``, ``FusedAdam`` flattening) recaptures.

Set ``MER_GRAPHS=0`` to run every launch eagerly (A/B and debugging).
"""
from __future__ import annotations

import contextlib
import gc
import os
from typing import Callable, Dict, Optional

import torch

ENABLED = os.environ.get("MER_GRAPHS", "1") != "0"
WARMUP_CALLS = 1  # eager calls per key before capturing (first-call caches: packed weights, bucket table)


class StaticGraph:
    """``fn(*static_inputs)`` captured once; ``replay(*inputs)`` copies inputs in and replays."""

    def __init__(self, fn: Callable, example_inputs, stream: Optional[torch.cuda.Stream] = None):
        # Static buffers and the capture are made outside inference mode even when the caller runs under
        # torch.inference_mode() (the batch-inference runtime): inference tensors cannot be updated in place
        # later by a replay's input copy, nor can the CUDA generator's graph-safe state tensors that the
        # first capture of the process creates.
        # No garbage collection while capturing: a collected cycle holding an older graph (or its memory pool)
        # would destroy it mid-capture, which HIP refuses ("operation not permitted when stream is capturing")
        # from inside a destructor -- an abort, not an exception.
        was_enabled = gc.isenabled()
        with torch.inference_mode(False):
            self.static_in = [t.detach().clone() for t in example_inputs]
            self.graph = torch.cuda.CUDAGraph()
            cur = stream if stream is not None else torch.cuda.current_stream()
            side = torch.cuda.Stream(device=cur.device)
            side.wait_stream(cur)
            gc.collect()
            gc.disable()
            try:
                with torch.cuda.graph(self.graph, stream=side):
                    self.out = fn(*self.static_in)
            finally:
                if was_enabled:
                    gc.enable()
            cur.wait_stream(side)

    def replay(self, *inputs):
        for st, x in zip(self.static_in, inputs):
            if st.data_ptr() != x.data_ptr():
                with torch.inference_mode(False):
                    st.copy_(x)
        self.graph.replay()
        return self.out


_BORROW = [0]
_BORROWED = set()  # storage addresses of static outputs handed out without a copy


@contextlib.contextmanager
def borrow_outputs():
    """Inside this context, graph outputs are handed out as the graph's static tensors themselves (no copy).
    For a caller that consumes them before the graph's next replay -- FusionModel feeding the encoders' outputs
    to the head graph, which copies them into its own static inputs -- this removes one device copy per output
    per step.  Outside it every output is a fresh copy (a caller may hold it across replays)."""
    _BORROW[0] += 1
    try:
        yield
    finally:
        _BORROW[0] -= 1


def hand_out(t: torch.Tensor) -> torch.Tensor:
    """A captured graph's static output for the caller: the tensor itself inside ``borrow_outputs()``, else a
    copy."""
    if _BORROW[0]:
        _BORROWED.add(t.untyped_storage().data_ptr())
        return t
    return t.clone()


def is_borrowed(t: torch.Tensor) -> bool:
    """True when ``t`` shares storage with a graph output handed out by ``hand_out`` without a copy (it is
    overwritten by that graph's next replay)."""
    return isinstance(t, torch.Tensor) and t.is_cuda and t.untyped_storage().data_ptr() in _BORROWED


class GraphCache:
    """Per-key call counter + captured graphs (eager for the first WARMUP_CALLS calls of a key)."""

    def __init__(self):
        self.calls: Dict[tuple, int] = {}
        self.graphs: Dict[tuple, object] = {}

    def ready(self, key) -> bool:
        """True when ``key`` should run through a (possibly not yet captured) graph."""
        if not ENABLED:
            return False
        n = self.calls.get(key, 0)
        self.calls[key] = n + 1
        return n >= WARMUP_CALLS

    def get(self, key):
        return self.graphs.get(key)

    def put(self, key, g):
        # keep one graph per shape family: drop graphs whose weight addresses are stale
        for k in [k for k in self.graphs if k[:-1] == key[:-1] and k != key]:
            del self.graphs[k]
        self.graphs[key] = g
        return g


class PendingGuard:
    """Bookkeeping for a captured forward graph whose static activations a later backward graph reads.

    ``claim()`` marks a forward as in flight (returns its generation); a second forward while one is in
    flight must run eagerly.  The in-flight mark is released by the backward (``release(gen)``) or, when the
    forward's autograd graph is dropped without a backward (a modality cut by ModalityDropout, an evaluation
    forward under grad mode), by the token the forward stored in its autograd context."""

    def __init__(self):
        self.pending = 0
        self._gen = 0

    def claim(self, want_backward: bool) -> int:
        self._gen += 1
        if want_backward:
            self.pending = self._gen
        return self._gen

    def release(self, gen: int) -> None:
        if self.pending == gen:
            self.pending = 0

    def token(self, gen: int):
        return _PendingToken(self, gen)


class _PendingToken:
    def __init__(self, guard: PendingGuard, gen: int):
        self.guard, self.gen = guard, gen

    def __del__(self):
        self.guard.release(self.gen)


def module_tensors(module: torch.nn.Module) -> list:
    """Every parameter and buffer of ``module``, listed once per module (the module tree is fixed after
    construction; tensors are re-homed in place by .to() / FusedAdam, so the Python objects stay valid)."""
    lst = module.__dict__.get("_mer_tensor_list")
    if lst is None:
        lst = list(module.parameters()) + list(module.buffers())
        module.__dict__["_mer_tensor_list"] = lst
    return lst


def tensor_addresses(module: torch.nn.Module) -> tuple:
    """Device addresses of every parameter and buffer (part of a graph key)."""
    return tuple(t.data_ptr() for t in module_tensors(module))


def capturing() -> bool:
    return torch.cuda.is_current_stream_capturing()
