"""Data parallelism over RCCL (torch.distributed 'nccl' backend == RCCL on ROCm), one process per GPU.

The reference has no distributed code; this is the north star's DP layer:
every rank runs the full train step on its own B=32 slice (weak scaling), BatchNorm keeps per-replica
batch statistics (no SyncBN, like the reference's single-GPU semantics), and the only exchange is a
SUM all-reduce of the flat fp32 gradient buffer owned by ``FusedAdam`` -- bucketed so each RCCL call
moves a few tens of MB (xGMI rings are per-link bound; fewer, larger collectives win), with the
1/world_size averaging folded into the Adam kernel (``grad_scale``) instead of an extra pass.
"""
from __future__ import annotations

import os
from typing import List

import torch
import torch.distributed as dist

BUCKET_BYTES = 32 << 20


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


def buckets(flat: torch.Tensor, bucket_bytes: int = BUCKET_BYTES) -> List[torch.Tensor]:
    n = max(1, bucket_bytes // flat.element_size())
    return [flat[i:i + n] for i in range(0, flat.numel(), n)]


class GradAllReduce:
    """SUM all-reduce of the optimizer's flat gradient buckets; Adam then applies 1/world."""

    def __init__(self, optimizer, bucket_bytes: int = BUCKET_BYTES):
        self.opt = optimizer
        self.bucket_bytes = bucket_bytes
        self.world = dist.get_world_size() if is_dist() else 1
        optimizer.grad_scale = 1.0 / self.world

    def __call__(self) -> None:
        if self.world == 1:
            return
        for flat in self.opt.flat_grads():
            for b in buckets(flat, self.bucket_bytes):
                dist.all_reduce(b, op=dist.ReduceOp.SUM)


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Make every replica start from rank 0's parameters and buffers."""
    if not is_dist():
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src)
