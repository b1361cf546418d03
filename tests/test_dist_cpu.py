"""Data-parallel layer on CPU: world_size 2 over gloo (the GPU path uses the same code over RCCL).

Covers dist.GradAllReduce on the real FusedAdam flat buffers (optimizer construction runs on CPU; only
its step needs the HIP kernel): bucketed SUM all-reduce, the early (head + layer4) bucket launched from the
backward hook without being reduced twice, gradients produced outside the flat buffer (gather_grads), the
"has a gradient" union over ranks, rank-0 broadcast of parameters and buffers, and the max-over-ranks timing.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(worker, world=2, *extra):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))


def _two_layer(rank):
    torch.manual_seed(100 + rank)  # rank-dependent init: broadcast must make them equal
    return torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.Linear(32, 5))


def _worker_sum(rank, world, port, q):
    _env(rank, world, port)
    from multimodalemotionrecognition_amd.dist import GradAllReduce, broadcast_module, init_distributed
    from multimodalemotionrecognition_amd.optim import FusedAdam

    try:
        w, r, _ = init_distributed(backend="gloo")
        assert (w, r) == (world, rank)
        m = _two_layer(rank)
        opt = FusedAdam(list(m.parameters()))
        ar = GradAllReduce(opt, bucket_bytes=1024, model=m, mask_sync=True)  # broadcasts rank 0's weights
        (g,) = opt.flat_grads()
        g.copy_(torch.arange(g.numel(), dtype=torch.float32) * (rank + 1))
        ar()
        expect = torch.arange(g.numel(), dtype=torch.float32) * sum(range(1, world + 1))
        ok_sum = torch.equal(g, expect)
        ok_scale = abs(opt.grad_scale - 1.0 / world) < 1e-12
        ref0 = _two_layer(0)
        ok_bcast = all(torch.equal(a, b) for a, b in zip(m.parameters(), ref0.parameters()))
        m2 = torch.nn.Linear(4, 3)
        with torch.no_grad():
            m2.weight.fill_(float(rank))
        broadcast_module(m2)
        ok_bcast = ok_bcast and bool(torch.all(m2.weight == 0.0))
        t = torch.tensor([float(rank + 1)])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
        q.put((rank, ok_sum, ok_scale, ok_bcast, float(t)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_grad_allreduce_world2_gloo():
    for rank, ok_sum, ok_scale, ok_bcast, tmax in _run(_worker_sum):
        assert ok_sum and ok_scale and ok_bcast, (rank, ok_sum, ok_scale, ok_bcast)
        assert tmax == 2.0


def _worker_early_bucket(rank, world, port, q, hook_ranks=(0, 1)):
    """A real (CPU autograd) backward: the first layer's grads are announced early through grads_ready (the
    trunk hook's role), the rest go at __call__; autograd produced every .grad OUTSIDE the flat buffer, so the
    hook itself must bring the prefix home before launching (then gather_grads the rest).  Ranks not in
    ``hook_ranks`` never see the hook (gated ModalityDropout detaching the video branch): they must issue the
    same prefix bucket at __call__ -- same boundaries, no hang.  Every element must be reduced exactly once."""
    _env(rank, world, port)
    from multimodalemotionrecognition_amd.dist import GradAllReduce, init_distributed
    from multimodalemotionrecognition_amd.optim import FusedAdam

    try:
        init_distributed(backend="gloo")
        m = _two_layer(0)
        head, tail = list(m[1].parameters()), list(m[0].parameters())
        opt = FusedAdam(head + tail)  # backward order: the last layer first (the early bucket's prefix)
        ar = GradAllReduce(opt, bucket_bytes=256, mask_sync=True, early_params=head)
        early_end = dict(ar._early_end)
        for it in range(2):
            opt.zero_grad()
            x = torch.randn(8, 64, generator=torch.Generator().manual_seed(rank + 10 * it))
            m(x).square().sum().backward()
            local = [p.grad.clone() for p in head + tail]
            if rank in hook_ranks:
                ar.grads_ready()      # BEFORE gather_grads: the hook homes the prefix itself
            ar()
            tot = [t.clone() for t in local]
            for t in tot:
                dist.all_reduce(t)
            ok = all(torch.allclose(p.grad, t, rtol=0, atol=1e-6) for p, t in zip(head + tail, tot))
            (g,) = opt.flat_grads()
            ok_flat = all(p.grad.data_ptr() == g[o:].data_ptr() for _, p, o, _ in opt.param_slices())
            if not (ok and ok_flat):
                break
        q.put((rank, ok, ok_flat, early_end.get(0, 0), None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("hook_ranks", [(0, 1), (0,), ()])
def test_early_bucket_and_gather_world2_gloo(hook_ranks):
    for rank, ok, ok_flat, early, _ in _run(_worker_early_bucket, 2, hook_ranks):
        assert ok and ok_flat, (rank, ok, ok_flat)
        # head = Linear(32, 5): weight 160 + bias 5 (padded to 8) = 168 flat elements in the early prefix
        assert early == 168, early


def _worker_used_union(rank, world, port, q):
    """ModalityDropout-style: a parameter has no gradient on rank 0 but has one on rank 1 -> both ranks must
    treat it as updated (union), with the all-reduced value in its slot."""
    _env(rank, world, port)
    from multimodalemotionrecognition_amd.dist import GradAllReduce, init_distributed
    from multimodalemotionrecognition_amd.optim import FusedAdam

    try:
        init_distributed(backend="gloo")
        a, b, c = torch.nn.Linear(4, 4), torch.nn.Linear(4, 4), torch.nn.Linear(4, 4)
        opt = FusedAdam(list(a.parameters()) + list(b.parameters()) + list(c.parameters()))
        ar = GradAllReduce(opt, mask_sync=True)
        opt.zero_grad()
        from multimodalemotionrecognition_amd.fusion import grad_buffer
        for p in a.parameters():
            p.grad = grad_buffer(p).fill_(1.0)
        if rank == 1:
            for p in b.parameters():
                p.grad = grad_buffer(p).fill_(2.0)
        ar()
        used = opt._used[0]
        b_vals = [float(p.grad.mean()) if p.grad is not None else float(grad_buffer(p).mean()) for p in b.parameters()]
        q.put((rank, used, b_vals))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_used_union_world2_gloo():
    for rank, used, b_vals in _run(_worker_used_union):
        assert used == [True, True, True, True, False, False], (rank, used)
        assert b_vals == [2.0, 2.0], (rank, b_vals)


def test_single_process_is_noop():
    from multimodalemotionrecognition_amd.dist import GradAllReduce, is_dist
    from multimodalemotionrecognition_amd.optim import FusedAdam

    assert not is_dist()
    m = torch.nn.Linear(4, 2)
    opt = FusedAdam(list(m.parameters()))
    (g,) = opt.flat_grads()
    g.fill_(1.0)
    GradAllReduce(opt)()
    assert torch.equal(g, torch.ones_like(g)) and opt.grad_scale == 1.0


def test_fused_adam_per_param_steps_and_order():
    """torch Adam keeps one step count per parameter: a parameter without a gradient is not counted (its bias
    correction lags).  FusedAdam's run planning (no HIP launch here: zero runs are planned when nothing has a
    gradient) tracks that."""
    from multimodalemotionrecognition_amd.optim import FusedAdam

    m = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 4))
    opt = FusedAdam(list(m.parameters()))
    opt.zero_grad()
    opt.set_used([[False, False, False, False]])
    opt.step()
    assert opt.state_steps() == [[0, 0, 0, 0]]


def test_optimizer_excludes_unused_and_orders_for_backward():
    """only the used trainables (ResNet18 11,176,512 + xattn head 381,064) are optimised and
    all-reduced; the flat layout starts with the head, then layer4, and ends with the stem."""
    from multimodalemotionrecognition_amd.train import build_model, build_optimizer_param_order

    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True)
    names = {id(q): n for n, q in m.named_parameters()}
    order = [names[id(q)] for q in build_optimizer_param_order(m)]
    assert sum(dict(m.named_parameters())[n].numel() for n in order) == 11_557_576
    assert not any(n.startswith(("audio_time_conv", "audio_model.classifier", "video_model.classifier")) for n in order)
    first_trunk = next(i for i, n in enumerate(order) if n.startswith("video_model.backbone."))
    assert all(not n.startswith(("video_model.", "audio_model.")) for n in order[:first_trunk])
    assert order[first_trunk].startswith("video_model.backbone.7.1.")
    assert order[-1].startswith("video_model.backbone.1.") and order[-3] == "video_model.backbone.0.weight"
    assert m.may_skip_grads() is False
    g = build_model(8, "gated", pretrained_video=False, use_wavlm=True)
    assert g.may_skip_grads() is True
