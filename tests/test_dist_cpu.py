"""Data-parallel layer on CPU: world_size 2 over gloo (the GPU path uses the same code over RCCL)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


class _FakeOpt:
    """Stands in for FusedAdam: exposes flat gradient buffers and a grad_scale slot."""

    def __init__(self, flats):
        self._f = flats
        self.grad_scale = 1.0

    def flat_grads(self):
        return self._f


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from multimodalemotionrecognition_amd.dist import GradAllReduce, broadcast_module, buckets, init_distributed

    try:
        w, r, _ = init_distributed(backend="gloo")
        assert (w, r) == (world, rank)
        # gradients differ per rank; after the SUM all-reduce every rank holds the same sum, and the
        # optimizer is told to average (grad_scale = 1/world)
        g = torch.arange(10_000, dtype=torch.float32) * (rank + 1)
        opt = _FakeOpt([g])
        ar = GradAllReduce(opt, bucket_bytes=4096)  # many buckets
        ar()
        expect = torch.arange(10_000, dtype=torch.float32) * sum(range(1, world + 1))
        ok_sum = torch.equal(g, expect)
        ok_scale = abs(opt.grad_scale - 1.0 / world) < 1e-12
        nb = len(buckets(g, 4096))
        m = torch.nn.Linear(4, 3)
        with torch.no_grad():
            m.weight.fill_(float(rank))
        broadcast_module(m)
        ok_bcast = bool(torch.all(m.weight == 0.0))
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
        q.put((rank, ok_sum, ok_scale, nb, ok_bcast, float(t)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_allreduce_world2_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=10) for _ in range(world))
    for p in procs:
        assert p.exitcode == 0
    for rank, ok_sum, ok_scale, nb, ok_bcast, tmax in res:
        assert ok_sum and ok_scale and ok_bcast, (rank, ok_sum, ok_scale, ok_bcast)
        assert nb == 10  # 40 KB of fp32 in 4 KB buckets
        assert tmax == float(world)


def test_single_process_is_noop():
    from multimodalemotionrecognition_amd.dist import GradAllReduce, is_dist

    assert not is_dist()
    g = torch.ones(8)
    opt = _FakeOpt([g])
    GradAllReduce(opt)()
    assert torch.equal(g, torch.ones(8)) and opt.grad_scale == 1.0


def _worker_groups(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from multimodalemotionrecognition_amd.dist import GradAllReduce, init_distributed
    from multimodalemotionrecognition_amd.optim import FusedAdam

    try:
        init_distributed(backend="gloo")
        torch.manual_seed(0)
        a, b = torch.nn.Linear(8, 4), torch.nn.Linear(6, 3)
        # stage-2 style param groups (train.py:831-872): one flat gradient buffer per group, all all-reduced
        opt = FusedAdam([{"params": list(a.parameters()), "lr": 1e-3}, {"params": list(b.parameters()), "lr": 1e-5}])
        flats = opt.flat_grads()
        for i, f in enumerate(flats):
            f.copy_(torch.arange(f.numel(), dtype=torch.float32) * (rank + 1) + i)
        GradAllReduce(opt, bucket_bytes=64)()
        # sum over ranks of arange * (rank + 1) + i
        ok = all(torch.equal(f, torch.arange(f.numel(), dtype=torch.float32) * sum(range(1, world + 1)) + i * world)
                 for i, f in enumerate(flats))
        q.put((rank, ok, len(flats), abs(opt.grad_scale - 1.0 / world) < 1e-12))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_allreduce_stage_groups_world2_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_groups, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    res = sorted(q.get(timeout=10) for _ in range(world))
    for p in procs:
        assert p.exitcode == 0
    for rank, ok, ngroups, ok_scale in res:
        assert ok and ngroups == 2 and ok_scale, (rank, ok, ngroups, ok_scale)
