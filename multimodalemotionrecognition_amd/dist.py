"""Data parallelism over RCCL (torch.distributed 'nccl' backend == RCCL on ROCm), one process per GPU.

The reference has no distributed code; this is the north star's DP layer
(SURVEY.md section 8(e)): every rank runs the full train step on its own B=32 slice (weak scaling),
BatchNorm keeps per-replica batch statistics (no SyncBN, like the reference's single-GPU semantics),
and the only data-path exchange is a SUM all-reduce of ``FusedAdam``'s flat fp32 gradient buffers.

* Only the USED trainables are in those buffers (``train.build_optimizer`` leaves out parameters the
  selected fusion mode never reaches, e.g. ``audio_time_conv`` and the encoders' classifiers under
  xattn), so no zeros cross xGMI.
* The buffers are laid out in backward order (head first, then ResNet18 layer4, layer3, ...): the
  bucket holding the head + layer4 gradients (~35 MB of the 46 MB) is launched as soon as the trunk's
  layer4 backward has been enqueued (``ResNet18Trunk`` calls the registered ready-hook between its two
  backward graphs), so its all-reduce runs on RCCL's stream while layer3..stem are still computing;
  the remaining ~11 MB go out after the backward.  1/world_size is folded into the Adam kernel
  (``grad_scale``) instead of an extra pass.
* Which parameters count as "having a gradient" this step is the union over ranks (gated-mode
  ModalityDropout and stage-2 LayerDrop leave some ``.grad`` None on some ranks): a host-side
  all-reduce of the per-parameter flags over a gloo group, as DDP does for unused parameters --
  host-to-host only, the GPU queue is not synchronised.
"""
from __future__ import annotations

import os
import time
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20
_CPU_GROUP = None


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str = None):
    """Initialise the process group from torchrun env vars (no-op for a single process)."""
    world, rank, local = env_world()
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return world, rank, local


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def cpu_group():
    """A gloo group over the same ranks for small host-side collectives (created once, by every rank at the
    same point: GradAllReduce's constructor).  Always a group of its OWN, even under a gloo default backend:
    collectives on one group are matched by issue order, and the early gradient bucket may be issued before
    (hook fired) or after (hook did not fire) the flag all-reduce on different ranks."""
    global _CPU_GROUP
    if _CPU_GROUP is None:
        _CPU_GROUP = dist.new_group(backend="gloo")
    return _CPU_GROUP


def buckets(flat: torch.Tensor, bucket_bytes: int = BUCKET_BYTES) -> List[torch.Tensor]:
    n = max(1, bucket_bytes // flat.element_size())
    return [flat[i:i + n] for i in range(0, flat.numel(), n)]


def _ranges(lo: int, hi: int, n: int) -> List[Tuple[int, int]]:
    return [(i, min(hi, i + n)) for i in range(lo, hi, n)]


class CommTimes:
    """Per-step diagnostics of the gradient all-reduce schedule (bench.py's ``dp`` fields), recorded when
    ``GradAllReduce(timing=True)``: marks on the compute stream (HIP events; host clock for a CPU / gloo run) at

    * ``hook``: the early bucket's launch point (layer4's backward enqueued, ``grads_ready``),
    * ``bwd_end``: ``__call__`` entry -- the whole backward is enqueued before it, so on the GPU the event completes
      when the backward has finished,
    * ``wait0`` / ``wait1``: around the waits on the launched collectives (for RCCL ``wait()`` makes the compute
      stream wait for RCCL's stream, so wait0 -> wait1 is the communication the step could not hide).

    ``summary()`` (after a device synchronise): per-step means of ``exposed_ms`` = wait0 -> wait1 and
    ``early_lead_ms`` = hook -> bwd_end (how long before the backward's end the early bucket went out)."""

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.steps, self.cur = [], {}

    def mark(self, name: str) -> None:
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.cur[name] = e
        else:
            self.cur[name] = time.perf_counter()

    def end_step(self) -> None:
        self.steps.append(self.cur)
        self.cur = {}

    def reset(self) -> None:
        self.steps, self.cur = [], {}

    def _ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.cuda else (b - a) * 1e3

    def summary(self) -> dict:
        exp = [self._ms(s["wait0"], s["wait1"]) for s in self.steps if "wait0" in s and "wait1" in s]
        lead = [self._ms(s["hook"], s["bwd_end"]) for s in self.steps if "hook" in s and "bwd_end" in s]
        mean = (lambda v: round(sum(v) / len(v), 4) if v else None)
        return {"steps": len(self.steps), "allreduce_exposed_ms": mean(exp), "early_bucket_lead_ms": mean(lead),
                "early_bucket_steps": len(lead)}


class GradAllReduce:
    """Bucketed SUM all-reduce of the optimizer's flat gradient buffers; Adam then applies 1/world.

    ``model``: when given, parameters and buffers are broadcast from rank 0 once (identical replicas
    before step 0), and the model's early-gradient hook (``register_grad_ready_hook``) is used to start
    the head + layer4 bucket while the rest of the backward runs.  ``mask_sync``: union the per-parameter
    "has a gradient" flags over ranks (default: ask the model whether some step can leave a trainable
    parameter without a gradient).

    Bucket boundaries never depend on the rank or the step: the early prefix ``[0, E)`` of each flat buffer is
    fixed at construction from the STATIC set of parameters the hook announces (``model.early_grad_params()``
    or ``early_params``).  A rank whose hook did not fire this step (gated ModalityDropout dropping the video
    branch detaches it, so the trunk backward never runs) launches ``[0, E)`` at ``__call__`` with the same
    chunking, before ``[E, N)``: every rank issues the same sequence of collectives."""

    def __init__(self, optimizer, bucket_bytes: int = BUCKET_BYTES, model: Optional[torch.nn.Module] = None,
                 mask_sync: Optional[bool] = None, early_params=None, force: bool = False, timing: bool = False):
        """``force``: run the bucket / hook / collective path even in a world of one process (an initialised
        1-rank group: the RCCL wiring test on a single GPU; the sums are identities).  ``timing``: record
        ``CommTimes`` marks every step (``self.times``)."""
        self.opt = optimizer
        self.times = None
        if timing:
            flat = optimizer.flat_grads()
            self.times = CommTimes(bool(flat) and flat[0].is_cuda)
        self.bucket_bytes = bucket_bytes
        self.world = dist.get_world_size() if is_dist() else 1
        self.active = self.world > 1 or (force and dist.is_available() and dist.is_initialized())
        optimizer.grad_scale = 1.0 / self.world
        self._pending = []      # async works launched this step
        self._done = {}         # group index -> flat elements already launched (the early prefix)
        if mask_sync is None:
            mask_sync = bool(getattr(model, "may_skip_grads", lambda: True)()) if model is not None else True
        self.mask_sync = mask_sync
        if mask_sync and self.active:
            cpu_group()
        if model is not None and self.active:
            broadcast_module(model)
            with torch.no_grad():  # re-homed trainables: one broadcast per flat buffer
                for f in optimizer.flat_params():
                    dist.broadcast(f, 0)
        if early_params is None and model is not None and hasattr(model, "early_grad_params"):
            early_params = model.early_grad_params()
        self._early_ids = {id(p) for p in (early_params or [])}
        self._early_end = self._prefix_ends(self._early_ids)
        if self._early_end and model is not None and hasattr(model, "register_grad_ready_hook"):
            model.register_grad_ready_hook(self.grads_ready)

    def _prefix_ends(self, ids) -> dict:
        """Per flat buffer: the end of the longest prefix made of parameters in ``ids`` (0 entries dropped)."""
        ends, stopped = {}, set()
        for gi, p, o, n in self.opt.param_slices():
            if gi in stopped:
                continue
            if id(p) in ids:
                ends[gi] = o + (n + 3) // 4 * 4
            else:
                stopped.add(gi)
        return {gi: e for gi, e in ends.items() if e > 0}

    def _launch(self, gi: int, flat: torch.Tensor, lo: int, hi: int) -> None:
        n = max(1, self.bucket_bytes // flat.element_size())
        for a, b in _ranges(lo, hi, n):
            self._pending.append(dist.all_reduce(flat[a:b], op=dist.ReduceOp.SUM, async_op=True))

    @torch.no_grad()
    def _home_prefix(self) -> None:
        """Copy any early-prefix gradient autograd produced OUTSIDE the flat buffer into its slot (enqueued before
        the collective on the same stream), so the early bucket never ships a stale slot that ``gather_grads``
        would overwrite while RCCL still reads it."""
        for gi, p, o, n in self.opt.param_slices():
            if id(p) not in self._early_ids or p.grad is None:
                continue
            flat = self.opt.flat_grads()[gi]
            if p.grad.data_ptr() != flat[o:].data_ptr():
                flat[o:o + n].view_as(p).copy_(p.grad)
                p.grad = flat[o:o + n].view_as(p)

    def grads_ready(self, params=None) -> None:
        """Early hook: the static early prefix has its final local gradients (enqueued on the current stream).
        Launches ``[0, E)`` of every flat buffer (once per step)."""
        if not self.active:
            return
        if self.times is not None:
            self.times.mark("hook")
        self._home_prefix()
        for gi, flat in enumerate(self.opt.flat_grads()):
            end, start = self._early_end.get(gi, 0), self._done.get(gi, 0)
            if end > start:
                self._launch(gi, flat, start, end)
                self._done[gi] = end

    def __call__(self) -> None:
        if self.times is not None and self.active:
            self.times.mark("bwd_end")
        used = self.opt.gather_grads()
        if not self.active:
            self._done = {}
            return
        if self.mask_sync:
            flags = torch.tensor([int(u) for g in used for u in g], dtype=torch.int32)
            dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=cpu_group())
            it = iter(flags.tolist())
            self.opt.set_used([[bool(next(it)) for _ in g] for g in used])
        for gi, flat in enumerate(self.opt.flat_grads()):
            end, start = self._early_end.get(gi, 0), self._done.get(gi, 0)
            if end > start:  # the hook did not fire on this rank this step: same prefix, same chunking
                self._launch(gi, flat, start, end)
            if max(end, start) < flat.numel():
                self._launch(gi, flat, max(end, start), flat.numel())
        if self.times is not None:
            self.times.mark("wait0")
        for w in self._pending:
            w.wait()
        if self.times is not None:
            self.times.mark("wait1")
            self.times.end_step()
        self._pending, self._done = [], {}


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every replica start from rank 0's parameters and buffers."""
    if not is_dist():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src)
