"""FusedAdam: ``torch.optim.Adam`` semantics (train.py:872,902) as ONE HIP kernel per contiguous run.

Each param group's parameters are re-homed into one flat fp32 buffer (``p.data`` becomes a
16-byte-aligned view), with a matching flat gradient buffer whose views the backward kernels
write into directly (``fusion.grad_buffer``), and flat ``exp_avg`` / ``exp_avg_sq`` state.
The flat gradient buffer is also what the data-parallel all-reduce ships (``dist.py``).

Like torch's Adam, parameters whose ``.grad`` is None are skipped (no moment decay, no weight
decay, no step increment), and the bias correction uses each parameter's OWN step count
(torch keeps ``state[p]['step']`` per parameter): the kernel runs over maximal runs of
adjacent params that have a gradient and share a step count.  With data parallelism the
"has a gradient" set is the union over ranks (``set_used``), as DDP does for parameters unused
on some ranks.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from . import kernels as K


def _align4(n: int) -> int:
    return (n + 3) // 4 * 4


def weight_version(p: torch.Tensor) -> tuple:
    """Identity of a weight's current VALUE for derived-copy caches (bf16 packs, INT8 images): storage
    address, autograd version counter, and the FusedAdam update count -- the Adam kernel writes the flat
    buffer through a raw pointer, which PyTorch's version counter never sees."""
    return (p.data_ptr(), p._version, getattr(p, "_mer_updates", 0))


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.grad_scale = 1.0  # set to 1/world_size by the data-parallel wrapper (SUM all-reduce)
        self._used: Optional[List[List[bool]]] = None  # set_used(): per-group per-param override for one step
        self._flat = []
        for group in self.param_groups:
            ps: List[torch.Tensor] = group["params"]
            if not ps:
                self._flat.append(None)
                continue
            dev = ps[0].device
            offs, total = [], 0
            for p in ps:
                if p.dtype != torch.float32:
                    raise TypeError("FusedAdam keeps fp32 master weights")
                offs.append(total)
                total += _align4(p.numel())
            flat = torch.zeros(total, device=dev, dtype=torch.float32)
            gflat = torch.zeros(total, device=dev, dtype=torch.float32)
            with torch.no_grad():
                for p, o in zip(ps, offs):
                    flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                    p.data = flat[o:o + p.numel()].view_as(p)
                    # (buffer, offset): a FRESH view is built per backward (fusion.grad_buffer) so autograd's
                    # AccumulateGrad can adopt it without a copy (a view we also kept alive would be cloned)
                    p._mer_grad_slot = (gflat, o)
            self._flat.append(dict(flat=flat, gflat=gflat, m=torch.zeros_like(flat), v=torch.zeros_like(flat),
                                   offs=offs, steps=[0] * len(ps)))

    def flat_grads(self):
        return [f["gflat"] for f in self._flat if f is not None]

    def flat_params(self):
        return [f["flat"] for f in self._flat if f is not None]

    def param_slices(self):
        """(flat-buffer index as in ``flat_grads()``, param, offset, numel) of every managed parameter, in
        flat-buffer order."""
        out = []
        for gi, (f, group) in enumerate((f, g) for f, g in zip(self._flat, self.param_groups) if f is not None):
            for p, o in zip(group["params"], f["offs"]):
                out.append((gi, p, o, p.numel()))
        return out

    def zero_grad(self, set_to_none: bool = True) -> None:
        self._used = None
        for f, group in zip(self._flat, self.param_groups):
            if f is None:
                continue
            f["gflat"].zero_()
            for p in group["params"]:
                p.grad = None

    @torch.no_grad()
    def gather_grads(self) -> List[List[bool]]:
        """Bring every gradient autograd produced outside the flat buffer home into it (so the data-parallel
        all-reduce sees it) and return the local per-group "has a gradient" flags."""
        used = []
        for f, group in zip(self._flat, self.param_groups):
            if f is None:
                used.append([])
                continue
            gflat = f["gflat"]
            flags = []
            for p, o in zip(group["params"], f["offs"]):
                has = p.grad is not None
                if has and p.grad.data_ptr() != gflat[o:].data_ptr():
                    gflat[o:o + p.numel()].view_as(p).copy_(p.grad)
                    p.grad = gflat[o:o + p.numel()].view_as(p)
                flags.append(has)
            used.append(flags)
        return used

    def set_used(self, used: Sequence[Sequence[bool]]) -> None:
        """Override, for the next ``step``, which parameters count as having a gradient (the union over
        data-parallel ranks); their flat-buffer slots hold the reduced gradient."""
        self._used = [list(u) for u in used]

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        used = self._used if self._used is not None else self.gather_grads()
        self._used = None
        for f, group, flags in zip(self._flat, self.param_groups, used):
            if f is None:
                continue
            ps, steps = group["params"], f["steps"]
            runs, cur = [], None
            for i, (p, o) in enumerate(zip(ps, f["offs"])):
                if not flags[i]:
                    cur = None
                    continue
                steps[i] += 1
                end = o + _align4(p.numel())
                if cur is not None and cur[1] == o and cur[2] == steps[i]:
                    cur[1] = end
                else:
                    cur = [o, end, steps[i]]
                    runs.append(cur)
                p._mer_updates = getattr(p, "_mer_updates", 0) + 1
            b1, b2 = group["betas"]
            for s, e, t in runs:
                K.adam_step(f["flat"][s:e], f["gflat"][s:e], f["m"][s:e], f["v"][s:e], group["lr"], b1, b2,
                            group["eps"], group["weight_decay"], t, self.grad_scale)
        return loss

    def state_steps(self) -> List[List[int]]:
        """Per-group per-parameter Adam step counts (torch's ``state[p]['step']``)."""
        return [list(f["steps"]) if f is not None else [] for f in self._flat]
