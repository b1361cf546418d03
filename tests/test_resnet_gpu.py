"""ResNet18 trunk on HIP (NHWC bf16 implicit-GEMM convs, train-mode BatchNorm) vs the fp32 CPU oracle.

The oracle's ResNet18 is a restatement of torchvision's topology (torchvision is absent here:
parity UNPINNED against the reference package itself).  Kernel-level checks compare
each conv against torch.nn.functional on the same bf16-rounded operands (tight), the whole trunk
against the oracle with bf16 tolerances (relative RMS, stated below).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import params, resnet18_ref

pytestmark = pytest.mark.gpu

REL_RMS_FEAT = 3e-2
REL_RMS_GRAD = 6e-2


def rel_rms(y, ref):
    y = y.detach().float().cpu()
    ref = ref.detach().float().cpu()
    return float((y - ref).pow(2).mean().sqrt() / ref.pow(2).mean().sqrt().clamp_min(1e-12))


def to_nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("N,H,C,Kc,R,stride,pad", [
    (2, 28, 64, 64, 3, 1, 1), (2, 28, 64, 128, 3, 2, 1), (2, 28, 64, 128, 1, 2, 0),
    (2, 7, 256, 512, 3, 2, 1), (3, 17, 16, 24, 3, 1, 1), (2, 30, 8, 64, 7, 2, 3)])
def test_conv_fwd_dgrad_wgrad_vs_torch(N, H, C, Kc, R, stride, pad):
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(0)
    x = torch.randn(N, C, H, H).bfloat16().float()
    w = (torch.randn(Kc, C, R, R) / (C * R * R) ** 0.5).bfloat16().float()
    x.requires_grad_(True)
    w.requires_grad_(True)
    y = F.conv2d(x, w, stride=stride, padding=pad)
    dy = torch.randn_like(y).bfloat16().float()
    y.backward(dy)
    Ho = y.shape[2]
    xd = to_nhwc(x.detach()).bfloat16().cuda()
    wp = torch.empty(Kc, R * R * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w.detach().cuda(), wp, C, False)
    yd = torch.empty(N, Ho, Ho, Kc, device="cuda", dtype=torch.bfloat16)
    stats = K.bn_stats_buffer(Kc, "cuda", N * Ho * Ho)
    K.conv_fwd(xd, wp, yd, stats, R, R, stride, pad)
    stats = stats.sum(0)  # per-row-tile partial rows
    yr = to_nhwc(y.detach())
    assert rel_rms(yd, yr) < 1e-2
    ys = yd.float().cpu()
    assert torch.allclose(stats[:, 0].cpu(), ys.sum((0, 1, 2)), rtol=1e-3, atol=1e-2)
    # dgrad
    wt = torch.empty(C, R * R * Kc, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w.detach().cuda(), wt, C, True)
    dxd = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
    K.conv_dgrad(to_nhwc(dy).bfloat16().cuda(), wt, dxd, R, R, stride, pad)
    assert rel_rms(dxd, to_nhwc(x.grad)) < 1e-2
    # wgrad (fp32 PyTorch layout, accumulated)
    dw = torch.zeros(Kc, C, R, R, device="cuda")
    K.conv_wgrad(xd, to_nhwc(dy).bfloat16().cuda(), dw, R, R, stride, pad)
    assert rel_rms(dw, w.grad) < 1e-2


def build_trunk(seed=0):
    from multimodalemotionrecognition_amd.video import ResNet18Trunk

    m = ResNet18Trunk()
    sd = m.state_dict()
    names = [(k, tuple(v.shape)) for k, v in sd.items()]
    assert sorted(("backbone." + k, s) for k, s in names) == sorted(resnet18_ref.param_shapes())
    new = {k: torch.from_numpy(params.init_tensor("backbone." + k, s, seed)) for k, s in names}
    m.load_state_dict(new)
    ref = {"backbone." + k: v.clone() for k, v in new.items()}
    return m.cuda(), ref


@pytest.mark.parametrize("layer,bi", [(4, 0), (5, 0), (7, 1)])
def test_single_block_forward_backward_vs_oracle(layer, bi):
    """One BasicBlock in isolation (same bf16 input, same upstream gradient) so bf16 errors do not compound:
    forward rel-RMS < 1.5e-2, input/param gradients rel-RMS < 3e-2."""
    from multimodalemotionrecognition_amd.video import block_backward, block_forward

    m, p = build_trunk()
    m.train(True)
    blk = m[layer][bi]
    cin = blk.conv1.weight.shape[1]
    hw = {4: 28, 5: 28, 6: 14, 7: 4}[layer] if bi == 0 else {4: 28, 5: 14, 6: 7, 7: 4}[layer]
    torch.manual_seed(layer * 10 + bi)
    x = torch.randn(8, cin, hw, hw).abs().bfloat16().float()
    prefix = f"backbone.{layer}.{bi}."
    for k in p:
        if k.startswith(prefix) and not k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            p[k].requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = resnet18_ref.basic_block(xr, p, prefix, blk.stride, training=True)
    out, sv = block_forward(m, blk, to_nhwc(x).bfloat16().cuda(), True)
    assert rel_rms(out, to_nhwc(ref.detach())) < 1.5e-2
    g = torch.randn_like(ref).bfloat16().float()
    grads = {}
    dxin, _ = block_backward(m, blk, sv, to_nhwc(g).bfloat16().cuda(), grads)
    torch.cuda.synchronize()
    # Reference backward evaluated at OUR forward activations (same ReLU masks, same batch statistics):
    # an fp32 forward flips ~1% of near-zero ReLU decisions vs a bf16 forward, which alone moves masked
    # gradients by ~10% rel-RMS -- that is precision, not a kernel property, so it is factored out here.
    ref_grads = ref_block_backward(blk, sv, g, prefix, p)
    errs = {"dx": rel_rms(dxin, ref_grads["dx"])}
    for n, q in blk.named_parameters():
        errs[n] = rel_rms(grads[id(q)], ref_grads[n])
    print(f"block {layer}.{bi} rel-rms:", {k: round(v, 4) for k, v in errs.items()})
    assert all(v < 2e-2 for v in errs.values()), errs


def ref_block_backward(blk, sv, g_nchw, prefix, p):
    """fp32 torch backward of one BasicBlock given the HIP forward's saved bf16 activations."""
    from torch.nn.grad import conv2d_input, conv2d_weight

    f = lambda t: t.detach().float().cpu().permute(0, 3, 1, 2).contiguous()  # noqa: E731  NHWC bf16 -> NCHW fp32
    xin, bc1, _, ba1, bc2, _, cd, _, out = sv
    g = g_nchw * (f(out) > 0)

    def bn_bwd(gm, x, gamma):
        mean = x.mean((0, 2, 3), keepdim=True)
        var = x.var((0, 2, 3), unbiased=False, keepdim=True)
        rstd = (var + 1e-5).rsqrt()
        xhat = (x - mean) * rstd
        dgamma = (gm * xhat).sum((0, 2, 3))
        dbeta = gm.sum((0, 2, 3))
        dx = gamma.view(1, -1, 1, 1) * rstd * (gm - gm.mean((0, 2, 3), keepdim=True)
                                               - xhat * (gm * xhat).mean((0, 2, 3), keepdim=True))
        return dx, dgamma, dbeta

    W1, W2 = p[prefix + "conv1.weight"].detach(), p[prefix + "conv2.weight"].detach()
    r = {}
    dc2, r["bn2.weight"], r["bn2.bias"] = bn_bwd(g, f(bc2), p[prefix + "bn2.weight"].detach())
    r["conv2.weight"] = conv2d_weight(f(ba1), W2.shape, dc2, stride=1, padding=1)
    da1 = conv2d_input(f(ba1).shape, W2, dc2, stride=1, padding=1) * (f(ba1) > 0)
    dc1, r["bn1.weight"], r["bn1.bias"] = bn_bwd(da1, f(bc1), p[prefix + "bn1.weight"].detach())
    r["conv1.weight"] = conv2d_weight(f(xin), W1.shape, dc1, stride=blk.stride, padding=1)
    dx = conv2d_input(f(xin).shape, W1, dc1, stride=blk.stride, padding=1)
    if cd is not None:
        Wd = p[prefix + "downsample.0.weight"].detach()
        dcd, r["downsample.1.weight"], r["downsample.1.bias"] = bn_bwd(g, f(cd), p[prefix + "downsample.1.weight"].detach())
        r["downsample.0.weight"] = conv2d_weight(f(xin), Wd.shape, dcd, stride=blk.stride)
        dx = dx + conv2d_input(f(xin).shape, Wd, dcd, stride=blk.stride)
    else:
        dx = dx + g
    r["dx"] = dx.permute(0, 2, 3, 1)
    return r


@pytest.mark.parametrize("training", [True, False])
def test_trunk_forward_backward_vs_oracle(training):
    m, p = build_trunk()
    m.train(training)
    video, _, _ = params.clip_inputs(1, frames=4, seed=41)
    x = torch.from_numpy(video[0])  # [4,3,112,112]
    for k in p:
        if p[k].dtype == torch.float32 and not k.endswith(("running_mean", "running_var")):
            p[k].requires_grad_(True)
    ref = resnet18_ref.resnet18_trunk(p, x, training=training)
    y = m(x.cuda())
    assert tuple(y.shape) == (4, 512, 1, 1)
    e = rel_rms(y, ref)
    print("trunk feat rel-rms", e)
    assert e < REL_RMS_FEAT
    if training:  # running stats updated like torch (momentum 0.1, unbiased var)
        for n in ("1.running_mean", "1.running_var", "7.1.bn2.running_var"):
            assert rel_rms(m.state_dict()[n], p["backbone." + n]) < 2e-2, n
        assert int(m.state_dict()["1.num_batches_tracked"]) == 1
    g = torch.randn(4, 512, 1, 1)
    ref.backward(g)
    y.backward(g.cuda())
    # End-to-end through 17 conv+BN layers the bf16 forward error flips ReLU masks and compounds in
    # BatchNorm backward (per-block isolation above is the tight check); here: direction agreement.
    cos = {}
    for n, q in m.named_parameters():
        a = q.grad.detach().float().cpu().reshape(-1)
        r = p["backbone." + n].grad.reshape(-1)
        cos[n] = float(torch.dot(a, r) / (a.norm() * r.norm()).clamp_min(1e-20))
    print("trunk grad cosine:", {k: round(v, 4) for k, v in cos.items()})
    bad = {k: v for k, v in cos.items() if v < 0.85}
    assert not bad, bad


def test_maxpool_avgpool_kernels():
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(0)
    x = torch.randn(2, 8, 9, 9).bfloat16().float().requires_grad_(True)
    y = F.max_pool2d(x, 3, 2, 1)
    dy = torch.randn_like(y).bfloat16().float()
    y.backward(dy)
    xd = to_nhwc(x.detach()).bfloat16().cuda()
    yd = torch.empty(2, 5, 5, 8, device="cuda", dtype=torch.bfloat16)
    arg = torch.empty(2, 5, 5, 8, device="cuda", dtype=torch.uint8)
    K.maxpool_fwd(xd, yd, arg)
    assert torch.equal(yd.float().cpu(), to_nhwc(y.detach()))
    dxd = torch.empty_like(xd)
    K.maxpool_bwd(to_nhwc(dy).bfloat16().cuda(), arg, dxd)
    assert rel_rms(dxd, to_nhwc(x.grad)) < 1e-2
    feats = torch.empty(2, 8, device="cuda")
    K.avgpool_fwd(xd, feats)
    assert torch.allclose(feats.cpu(), x.detach().mean((2, 3)), atol=1e-3)


@pytest.mark.parametrize("N,H,C,Kc,R,stride,pad", [
    (2, 28, 64, 64, 3, 1, 1), (2, 28, 64, 128, 3, 2, 1), (2, 28, 64, 128, 1, 2, 0),
    (2, 7, 256, 512, 3, 2, 1), (3, 17, 16, 24, 3, 1, 1), (2, 30, 8, 64, 7, 2, 3), (5, 14, 256, 256, 3, 1, 1)])
def test_conv_variants_bit_identical(N, H, C, Kc, R, stride, pad):
    """The glds-pipelined conv (variant 1) against the register-staged one (variant 0): same fragment
    order and K order, so fwd (incl. fused BN stats up to atomic order) and dgrad (incl. the masked residual)
    agree bit for bit."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(1)
    Ho = (H + 2 * pad - R) // stride + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Kc, C, R, R, device="cuda") / (C * R * R) ** 0.5)
    wp = torch.empty(Kc, R * R * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    wt = torch.empty(C, R * R * Kc, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    ys, sts = [], []
    for v in (0, 1, 2, 3, 4, 5):
        y = torch.empty(N, Ho, Ho, Kc, device="cuda", dtype=torch.bfloat16)
        st = K.bn_stats_buffer(Kc, "cuda", N * Ho * Ho)
        K.conv_fwd(x, wp, y, st, R, R, stride, pad, variant=v)
        ys.append(y)
        sts.append(st.sum(0))
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    assert all(torch.allclose(sts[0], st, rtol=1e-5, atol=1e-3) for st in sts[1:])
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    res = torch.randn(N, H, H, C, device="cuda").bfloat16()
    mask = torch.randn(N, H, H, C, device="cuda").bfloat16()
    dxs = []
    for v in (0, 1, 2, 3, 4, 5):
        dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        K.conv_dgrad(dy, wt, dx, R, R, stride, pad, residual=res, mask=mask, variant=v)
        dxs.append(dx)
    assert all(torch.equal(dxs[0], d) for d in dxs[1:])


@pytest.mark.parametrize("N", [3, 40, 256])
def test_halo_conv_bit_identical(N):
    """The layer1 halo kernel (variant 6: resident weights, per-tile input halo in LDS, persistent workgroups) against
    the pipelined implicit GEMM it replaces (fwd variant 2, dgrad variant 5): same fragments and K order -> identical
    outputs; the BN statistics and BN-backward sums (residual under a ReLU mask, two BNs), accumulated per persistent
    workgroup, agree to fp32 rounding once folded.  N = 3: a partial last tile; 40: fewer tiles than CUs; 256 (the B=32 step): ~6 tiles per
    workgroup, the double-buffered halo in use.  The default (-1) takes variant 6 on this shape."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(9)
    H, C = 28, 64
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = torch.randn(C, C, 3, 3, device="cuda") / 24.0
    wp = torch.empty(C, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    wt = torch.empty(C, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    outs = {}
    for v in (2, 6, -1):
        y = torch.full((N, H, H, C), float("nan"), device="cuda", dtype=torch.bfloat16)
        st = K.bn_stats_buffer(C, "cuda", N * H * H)
        K.conv_fwd(x, wp, y, st, 3, 3, 1, 1, variant=v)
        outs[v] = (y, st)
    # the halo kernel accumulates its BN statistics over each persistent workgroup's tiles (one partial row per
    # workgroup), so only the folded sums compare with the pipelined kernel's per-tile rows; repeatable bitwise
    for v in (6, -1):
        assert torch.equal(outs[2][0], outs[v][0]), v
        assert torch.allclose(outs[2][1].sum(0), outs[v][1].sum(0), rtol=1e-5, atol=1e-2), v
    assert torch.equal(outs[6][1], outs[-1][1])
    dy = torch.randn(N, H, H, C, device="cuda").bfloat16()
    res = torch.randn(N, H, H, C, device="cuda").bfloat16()
    mask = torch.randn(N, H, H, C, device="cuda").bfloat16()
    xb = torch.randn(N, H, H, C, device="cuda").bfloat16()
    xb2 = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ms = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    ms2 = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    rows = K.bn_red_rows(N * H * H)
    douts = {}
    for v in (5, 6, -1):
        dx = torch.full((N, H, H, C), float("nan"), device="cuda", dtype=torch.bfloat16)
        red = torch.zeros(rows, C, 2, device="cuda")
        red2 = torch.zeros(rows, C, 2, device="cuda")
        K.conv_dgrad(dy, wt, dx, 3, 3, 1, 1, residual=res, mask=mask, variant=v,
                     bnr=(mask, xb, ms, red, xb2, ms2, red2))
        douts[v] = (dx, red, red2)
    # dgrad: the halo kernel runs the forward's 8-wave layout (variant 5 has 4 waves), so the BN-backward partial rows
    # group their sums differently: dx bit-identical, the folded sums to fp32 rounding
    for v in (6, -1):
        assert torch.equal(douts[5][0], douts[v][0]), v
        for a, b in zip(douts[5][1:], douts[v][1:]):
            assert torch.allclose(a.sum(0), b.sum(0), rtol=1e-5, atol=1e-2), v
    assert torch.equal(douts[6][1], douts[-1][1]) and torch.equal(douts[6][2], douts[-1][2])
    # one fused BN (every layer1 dgrad of the train step): the halo kernel's instance without the second BN's sums
    one = {}
    for v in (5, 6):
        dx = torch.full((N, H, H, C), float("nan"), device="cuda", dtype=torch.bfloat16)
        red = torch.zeros(rows, C, 2, device="cuda")
        K.conv_dgrad(dy, wt, dx, 3, 3, 1, 1, residual=res, mask=mask, variant=v, bnr=(mask, xb, ms, red))
        one[v] = (dx, red)
    assert torch.equal(one[5][0], one[6][0]) and torch.equal(one[6][0], douts[6][0])
    assert torch.allclose(one[5][1].sum(0), one[6][1].sum(0), rtol=1e-5, atol=1e-2)
    assert torch.equal(one[6][1], douts[6][1])
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float(), padding=1).permute(0, 2, 3, 1)
    assert rel_rms(outs[6][0], ref) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N", [3, 40, 256])
def test_halo_partial_rows_fold(N):
    """K.conv_fwd / K.conv_dgrad return the partial rows their launch wrote (mer_conv_fwd_rows / mer_conv_dgrad_rows):
    one per persistent workgroup on the halo kernel (layer1; the stem), one per row tile otherwise.  Every row past
    the count is still zero, and the folds over the written rows alone (mer_bn_finalize_rows, mer_partials_sum) equal
    the folds over every row to fp32 rounding (the zero rows only change the fold's grouping)."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(19)

    def check_fwd(x, wp, Ho, R, pad, variants):
        C = wp.shape[0]
        M = x.shape[0] * Ho * Ho
        for v in variants:
            y = torch.empty(x.shape[0], Ho, Ho, C, device="cuda", dtype=torch.bfloat16)
            st = K.bn_stats_buffer(C, "cuda", M)
            rows = K.conv_fwd(x, wp, y, st, R, R, 1, pad, variant=v)
            tiles = K.bn_stat_rows(M) - 64
            if v == 2:
                assert rows == tiles
            else:
                assert 0 < rows <= -(-M // 128), (v, rows)
            assert not st[rows:].any()
            res = []
            for r in (rows, None):
                ms = torch.empty(C, 2, device="cuda")
                rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
                K.bn_finalize(st.clone(), M, 1e-5, 0.1, ms, rm, rv, rows=r)
                res.append(torch.cat([ms.flatten(), rm, rv]))
            assert torch.allclose(res[0], res[1], rtol=2e-6, atol=1e-6), v

    H, C = 28, 64
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = torch.randn(C, C, 3, 3, device="cuda") / 24.0
    wp = torch.empty(C, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    wt = torch.empty(C, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    check_fwd(x, wp, H, 3, 1, (2, 6, -1))
    # the stem's space-to-depth form: 4x4 / stride 1 / pad 0 on 16 channels, 59 -> 56
    xs = torch.randn(max(1, N // 8), 59, 59, 16, device="cuda").bfloat16()
    ws = torch.randn(C, 16, 4, 4, device="cuda") / 16.0
    wsp = torch.empty(C, 16 * 16, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(ws, wsp, 16, False)
    check_fwd(xs, wsp, 56, 4, 0, (6, -1))
    # the dgrad's fused BN-backward rows (one and two BNs)
    dy = torch.randn(N, H, H, C, device="cuda").bfloat16()
    res = torch.randn(N, H, H, C, device="cuda").bfloat16()
    mask = torch.randn(N, H, H, C, device="cuda").bfloat16()
    xb = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ms = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    M = N * H * H
    for v in (5, 6, -1):
        for two in (False, True):
            dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
            reds = [torch.zeros(K.bn_red_rows(M), C, 2, device="cuda") for _ in range(2)]
            bnr = (mask, xb, ms, reds[0]) + ((xb, ms, reds[1]) if two else ())
            rows = K.conv_dgrad(dy, wt, dx, 3, 3, 1, 1, residual=res, mask=mask, variant=v, bnr=bnr)
            if v == 5:
                assert rows == K.bn_red_rows(M) - 64
            else:
                assert 0 < rows <= -(-M // 128), (v, rows)
            for red in reds[:2 if two else 1]:
                assert not red[rows:].any()
                a = K.partials_sum(red.clone(), torch.empty(C, 2, device="cuda"), rows)
                b = K.partials_sum(red.clone(), torch.empty(C, 2, device="cuda"))
                assert torch.allclose(a, b, rtol=1e-5, atol=1e-3), (v, two)


@pytest.mark.parametrize("N", [3, 64])
def test_halo_stem_bit_identical(N):
    """The stem's space-to-depth form (4x4 / stride 1 / pad 0, 16 -> 64 channels, 59x59 -> 56x56) on the halo kernel
    (variant 6, two persistent workgroups per CU) against the pipelined implicit GEMM (variant 2): identical outputs
    (same 128 x 64 tiles, wave layout and epilogue), BN statistics to fp32 rounding once folded (accumulated per
    persistent workgroup); the default (-1) takes it."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(10)
    x = torch.randn(N, 59, 59, 16, device="cuda").bfloat16()
    w = torch.randn(64, 16, 4, 4, device="cuda") / 16.0
    wp = torch.empty(64, 256, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, 16, False)
    outs = {}
    for v in (2, 6, -1):
        y = torch.full((N, 56, 56, 64), float("nan"), device="cuda", dtype=torch.bfloat16)
        st = K.bn_stats_buffer(64, "cuda", N * 56 * 56)
        K.conv_fwd(x, wp, y, st, 4, 4, 1, 0, variant=v)
        outs[v] = (y, st)
    for v in (6, -1):
        assert torch.equal(outs[2][0], outs[v][0]), v
        assert torch.allclose(outs[2][1].sum(0), outs[v][1].sum(0), rtol=1e-5, atol=1e-2), v
    assert torch.equal(outs[6][1], outs[-1][1])
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float()).permute(0, 2, 3, 1)
    assert rel_rms(outs[6][0], ref) < 1e-2


@pytest.mark.parametrize("N,H,C,Kc,stride", [(8, 7, 256, 256, 1), (16, 4, 512, 512, 1), (8, 14, 128, 256, 2),
                                              (16, 7, 256, 512, 2), (5, 14, 128, 128, 1), (6, 28, 64, 64, 1),
                                              (3, 28, 64, 128, 2)])
@pytest.mark.parametrize("variant", [7])
def test_conv_split_k_groups(N, H, C, Kc, stride, variant):
    """In-workgroup split-K (variant 7: two K-groups of waves, each a contiguous half of the K-steps on its own LDS
    ring, tiles summed in group order in LDS) against the one-group kernel (variant 2) on the same tiles: the only
    difference is where the fp32 sum splits, so outputs agree to one bf16 rounding and the fused BN statistics /
    BN-backward sums (two BNs, residual under a ReLU mask, the stride-2 parity classes and the fused downsample
    segment) to fp32 rounding; every launch is bitwise repeatable.  Also against torch."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(11)
    Ho = (H + 2 - 3) // stride + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = torch.randn(Kc, C, 3, 3, device="cuda") / (9 * C) ** 0.5
    wp = torch.empty(Kc, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    wt = torch.empty(C, 9 * Kc, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    M, Mi = N * Ho * Ho, N * H * H

    def fwd(v):
        y = torch.full((N, Ho, Ho, Kc), float("nan"), device="cuda", dtype=torch.bfloat16)
        st = K.bn_stats_buffer(Kc, "cuda", M)
        K.conv_fwd(x, wp, y, st, 3, 3, stride, 1, variant=v)
        return y, st.sum(0)

    (y2, s2), (yk, sk), (yk2, sk2) = fwd(2), fwd(variant), fwd(variant)
    assert torch.equal(yk, yk2) and torch.equal(sk, sk2)
    assert rel_rms(yk, y2) < 4e-3
    assert (yk.float() - y2.float()).abs().max() <= 2 ** -6 * y2.float().abs().max()
    assert torch.allclose(sk, s2, rtol=1e-3, atol=0.5)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float(), stride=stride, padding=1).permute(0, 2, 3, 1)
    assert rel_rms(yk, ref) < 1e-2
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    mask = torch.randn(N, H, H, C, device="cuda").bfloat16()
    xb = torch.randn(N, H, H, C, device="cuda").bfloat16()
    xb2 = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ms = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    ms2 = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    kw = {}
    if stride == 2 and Kc % 64 == 0:  # the fused 1x1 / stride-2 downsample segment of parity class (0, 0)
        wd = torch.randn(Kc, C, 1, 1, device="cuda") / C ** 0.5
        wdt = torch.empty(C, Kc, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(wd, wdt, C, True)
        kw["ds"] = (torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16(), wdt)
    else:
        kw.update(residual=torch.randn(N, H, H, C, device="cuda").bfloat16(), mask=mask)

    def bwd(v, two):
        dx = torch.full((N, H, H, C), float("nan"), device="cuda", dtype=torch.bfloat16)
        rows = K.bn_red_rows(Mi)
        red, red2 = torch.zeros(rows, C, 2, device="cuda"), torch.zeros(rows, C, 2, device="cuda")
        bnr = (mask, xb, ms, red, xb2, ms2, red2) if two else (mask, xb, ms, red)
        K.conv_dgrad(dy, wt, dx, 3, 3, stride, 1, variant=v, bnr=bnr, **kw)
        return dx, red.sum(0), red2.sum(0)

    for two in (False, True):
        a, b, c = bwd(2, two), bwd(variant, two), bwd(variant, two)
        assert all(torch.equal(p, q) for p, q in zip(b, c))
        assert rel_rms(b[0], a[0]) < 4e-3
        for p, q in zip(a[1:], b[1:]):
            assert torch.allclose(p, q, rtol=1e-3, atol=0.5)


@pytest.mark.parametrize("stride,ds", [(1, False), (2, True)])
def test_dgrad_fused_bn_reduce_matches_standalone(stride, ds):
    """mer_conv_dgrad_bnr's epilogue reduction == mer_bn_bwd_reduce over the stored gradient (both BNs)."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(2)
    N, H, C, Kc = 4, 14, 64, 128
    Ho = (H + 2 - 3) // stride + 1
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    w = torch.randn(Kc, C, 3, 3, device="cuda") * 0.05
    wt = torch.empty(C, 9 * Kc, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    res = torch.randn(N, H, H, C, device="cuda").bfloat16()
    mask = torch.randn(N, H, H, C, device="cuda").bfloat16()
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    x2 = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ms = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    ms2 = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    rows = K.bn_red_rows(N * H * H)
    red_p = torch.zeros(rows, C, 2, device="cuda")
    red2_p = torch.zeros(rows, C, 2, device="cuda")
    dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
    bnr = (mask, x, ms, red_p, x2, ms2, red2_p) if ds else (mask, x, ms, red_p)
    K.conv_dgrad(dy, wt, dx, 3, 3, stride, 1, residual=res, mask=mask, bnr=bnr)
    dx_ref = torch.empty_like(dx)
    K.conv_dgrad(dy, wt, dx_ref, 3, 3, stride, 1, residual=res, mask=mask)
    assert torch.equal(dx, dx_ref)
    red = K.partials_sum(red_p, torch.empty(C, 2, device="cuda"))
    ref = torch.zeros(C, 2, device="cuda")
    K.bn_bwd_reduce(dx_ref, mask, x, ms, ref)
    assert torch.allclose(red, ref, rtol=1e-4, atol=1e-3)
    if ds:
        red2 = K.partials_sum(red2_p, torch.empty(C, 2, device="cuda"))
        ref2 = torch.zeros(C, 2, device="cuda")
        K.bn_bwd_reduce(dx_ref, mask, x2, ms2, ref2)
        assert torch.allclose(red2, ref2, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,H,C,Kc,R,stride,pad", [(2, 28, 64, 64, 3, 1, 1), (2, 14, 128, 256, 3, 2, 1),
                                                   (2, 30, 8, 64, 7, 2, 3), (4, 7, 512, 512, 3, 1, 1),
                                                   (32, 28, 64, 64, 3, 1, 1), (32, 28, 64, 128, 3, 2, 1),
                                                   (64, 14, 128, 256, 3, 1, 1), (64, 7, 256, 512, 1, 2, 0)])
def test_wgrad_variants_bit_identical(N, H, C, Kc, R, stride, pad):
    """Every wgrad variant gives the same bits: 4- / 8-wave register-staged (1, 2), 2-deep register prefetch (3),
    global_load_lds ring with 2 / 3 stages (4, 5) -- same pixel order per split, same split sum order."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(4)
    Ho = (H + 2 * pad - R) // stride + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    creal = 3 if C == 8 else C
    out = []
    for v in (1, 2, 3, 4, 5, 6, 7):
        dw = torch.zeros(Kc, creal, R, R, device="cuda")
        K.conv_wgrad(x, dy, dw, R, R, stride, pad, creal=creal, variant=v)
        out.append(dw)
    ref = (x.float().permute(0, 3, 1, 2)[:, :creal], dy.float().permute(0, 3, 1, 2))
    dw_ref = torch.nn.grad.conv2d_weight(ref[0], (Kc, creal, R, R), ref[1], stride=stride, padding=pad)
    assert (out[0] - dw_ref).abs().max() <= 5e-3 * dw_ref.abs().max() + 1e-3
    for v, o in zip((2, 3, 4, 5, 6, 7), out[1:]):
        assert torch.equal(out[0], o), f"variant {v} differs"


@pytest.mark.parametrize("N,H,C,Kc,R,stride,pad", [(2, 28, 64, 64, 3, 1, 1), (2, 14, 128, 256, 3, 2, 1),
                                                   (2, 30, 8, 64, 7, 2, 3), (4, 7, 512, 512, 3, 1, 1),
                                                   (32, 28, 64, 64, 3, 1, 1), (64, 14, 128, 256, 3, 1, 1),
                                                   (64, 7, 256, 512, 1, 2, 0), (256, 4, 512, 512, 3, 1, 1)])
def test_wgrad_split_k_groups(N, H, C, Kc, R, stride, pad):
    """The trunk's default weight gradient (variant 8: two K-groups of waves per workgroup, each a contiguous half of
    the split's pixels on its own ring, their tiles summed in LDS in group order) against the one-group ring (variant
    4) at the same split count: the fp32 sums split at a different place, so the two agree to fp32 rounding; every
    launch is bitwise repeatable (ragged splits included: P not a multiple of the split's 64-pixel steps)."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(12)
    Ho = (H + 2 * pad - R) // stride + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    creal = 3 if C == 8 else C
    P = N * Ho * Ho
    out = {}
    for v, splits in ((4, None), (8, None), (8, 3), (4, 3), (8, None)):
        dw = torch.zeros(Kc, creal, R, R, device="cuda")
        K.conv_wgrad(x, dy, dw, R, R, stride, pad, creal=creal, variant=v, splits=splits)
        out.setdefault((v, splits), []).append(dw)
    a, b = out[(8, None)]
    assert torch.equal(a, b)
    ref = (x.float().permute(0, 3, 1, 2)[:, :creal], dy.float().permute(0, 3, 1, 2))
    dw_ref = torch.nn.grad.conv2d_weight(ref[0], (Kc, creal, R, R), ref[1], stride=stride, padding=pad)
    scale = float(dw_ref.abs().max())
    for key in ((4, None), (8, None), (8, 3)):
        assert (out[key][0] - dw_ref).abs().max() <= 5e-3 * scale + 1e-3, key
    # same split count: only the in-workgroup split point differs
    assert (out[(8, 3)][0] - out[(4, 3)][0]).abs().max() <= 2e-5 * scale + 1e-6
    if P > 64:
        assert K.wgrad_split_count(P, 3) <= 3


def test_wgrad_fold_batch_matches_immediate_fold():
    """Deferred slabs folded by ONE mer_wgrad_fold_batch launch == the per-conv fold (fold+scatter below 17 slabs,
    reduce + scatter above), for records of 1-12, 13-48 and > 48 slabs, Creal < C, and the stem's map record
    (space-to-depth slabs gathered into the 7x7x3 weight); dw accumulates (+=) like the immediate path."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.video import S2D_CH, _stem_wgrad_index, _stem_wgrad_map

    torch.manual_seed(6)
    cases = [(2, 28, 64, 64, 3, 1, 1, None, 4), (4, 14, 128, 256, 3, 2, 1, None, 20),
             (32, 28, 64, 64, 3, 1, 1, None, 150), (2, 30, 8, 64, 7, 2, 3, 3, None), (8, 7, 256, 512, 1, 2, 0, None, None)]
    folds = K.WgradFolds()
    refs, outs, inits = [], [], []
    for N, H, C, Kc, R, stride, pad, creal, splits in cases:
        Ho = (H + 2 * pad - R) // stride + 1
        x = torch.randn(N, H, H, C, device="cuda").bfloat16()
        dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
        cr = creal or C
        init = torch.randn(Kc, cr, R, R, device="cuda")
        ref, out = init.clone(), init.clone()
        K.conv_wgrad(x, dy, ref, R, R, stride, pad, creal=cr, splits=splits)
        K.conv_wgrad(x, dy, out, R, R, stride, pad, creal=cr, splits=splits, defer=folds)
        refs.append(ref)
        outs.append(out)
        inits.append(init)
    # stem: 4x4 stride-1 wgrad on 16 space-to-depth channels, gathered to [64][3][7][7]
    xs = torch.randn(4, 31, 31, S2D_CH, device="cuda").bfloat16()
    dys = torch.randn(4, 28, 28, 64, device="cuda").bfloat16()
    ws = torch.zeros(64, S2D_CH, 4, 4, device="cuda")
    K.conv_wgrad(xs, dys, ws, 4, 4, 1, 0)
    w0 = torch.randn(64, 3, 7, 7, device="cuda")
    refs.append(w0 + ws.view(64, -1).index_select(1, _stem_wgrad_index(7, 7, 3, ws.device)).view(64, 3, 7, 7))
    out = w0.clone()
    K.conv_wgrad(xs, dys, out, 4, 4, 1, 0, defer=folds, dw_map=_stem_wgrad_map(7, 7, 3, out.device))
    outs.append(out)
    inits.append(w0)
    torch.cuda.synchronize()
    assert all(torch.equal(o, i) for o, i in zip(outs, inits))  # nothing folded before the flush
    folds.flush()
    for i, (r, o) in enumerate(zip(refs, outs)):
        assert (o - r).abs().max() <= 1e-5 * r.abs().max(), i


def test_trunk_backward_deferred_folds_match(monkeypatch):
    """The train step's trunk backward with deferred batched folds == with a fold after every wgrad (fp32
    summation order only), and bit-reproducible run to run."""
    from multimodalemotionrecognition_amd import video as V

    m, _ = build_trunk()
    m.train(True)
    video, _, _ = params.clip_inputs(1, frames=8, seed=44)
    x = torch.from_numpy(video[0]).cuda()
    res = []
    for defer in (False, True, True):
        monkeypatch.setattr(V, "WGRAD_DEFER", defer)
        f, saved = V.trunk_forward(m, x, True)
        g = V.trunk_backward(m, saved, torch.ones_like(f), True)
        res.append({k: v.clone() for k, v in g.items()})
        for q in m.parameters():
            q.grad = None
    for q in m.parameters():
        a, b, c = (r.get(id(q)) for r in res)
        if a is not None:
            assert torch.equal(b, c)
            assert (a - b).abs().max() <= 1e-5 * a.abs().max() + 1e-12


@pytest.mark.parametrize("H", [112, 32])
def test_space_to_depth_stem_vs_torch(H):
    """The stem conv (7x7, stride 2, pad 3) run as a 4x4 stride-1 conv on 2x2 space-to-depth frames:
    forward and weight gradient vs torch's conv2d on the same bf16-rounded operands."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.video import S2D_CH, _stem_wgrad_index

    torch.manual_seed(H)
    N = 2
    x = torch.randn(N, 3, H, H).bfloat16().float()
    w = (torch.randn(64, 3, 7, 7) / 147 ** 0.5).bfloat16().float()
    xs = torch.empty(N, H // 2 + 3, H // 2 + 3, S2D_CH, device="cuda", dtype=torch.bfloat16)
    K.pack_input_s2d(x.cuda(), xs)
    wd = w.cuda()
    wp = torch.empty(64, 4 * 4 * S2D_CH, device="cuda", dtype=torch.bfloat16)
    desc = torch.tensor([[wd.data_ptr(), wp.data_ptr(), 64, 3, 7, 7, S2D_CH, 2, 0]], dtype=torch.int64).cuda()
    K.pack_conv_weights(desc, 64)  # one block per output channel
    y = torch.empty(N, H // 2, H // 2, 64, device="cuda", dtype=torch.bfloat16)
    K.conv_fwd(xs, wp, y, None, 4, 4, 1, 0)
    wr = w.clone().requires_grad_(True)
    ref = F.conv2d(x, wr, stride=2, padding=3)
    assert rel_rms(y.float().permute(0, 3, 1, 2), ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    ws = torch.zeros(64, S2D_CH, 4, 4, device="cuda")
    K.conv_wgrad(xs, to_nhwc(dy).bfloat16().cuda(), ws, 4, 4, 1, 0)
    dw = ws.view(64, -1).index_select(1, _stem_wgrad_index(7, 7, 3, ws.device)).view(64, 3, 7, 7)
    assert rel_rms(dw, wr.grad) < 1e-2


def test_space_to_depth_pack_frame_chunks():
    """Above 2^22 packed pixels per launch (1204 frames at 112x112) the pack runs in frame chunks: the result
    equals per-frame-slice packs bit for bit (no batch-size ceiling from the index math)."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.video import S2D_CH

    N, H = 1300, 112
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(N, 3, H, H, device="cuda", generator=g)
    whole = torch.empty(N, H // 2 + 3, H // 2 + 3, S2D_CH, device="cuda", dtype=torch.bfloat16)
    K.pack_input_s2d(x, whole)
    part = torch.empty_like(whole)
    for n0 in range(0, N, 400):
        K.pack_input_s2d(x[n0:n0 + 400], part[n0:n0 + 400])
    torch.cuda.synchronize()
    assert torch.equal(whole.view(torch.int16), part.view(torch.int16))


@pytest.mark.parametrize("training", [True, False])
def test_fused_stem_tail_matches_unfused(training):
    """stem_bnrelu_maxpool == bn_apply(relu) -> maxpool_fwd bit for bit; stem_pool_bn_bwd == maxpool_bwd ->
    bn_bwd_reduce -> bn_bwd_apply (up to the fp32 atomic order of the channel sums)."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(5)
    N, H, C = 4, 56, 64
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    ms = torch.stack([torch.randn(C) * 0.1, torch.rand(C) + 0.5], 1).cuda().contiguous()
    g, b = (torch.rand(C) + 0.5).cuda(), (torch.randn(C) * 0.2).cuda()
    Hp = (H - 1) // 2 + 1
    a = torch.empty_like(x)
    K.bn_apply(x, ms, g, b, a, relu=True)
    p_ref = torch.empty(N, Hp, Hp, C, device="cuda", dtype=torch.bfloat16)
    arg_ref = torch.empty(N, Hp, Hp, C, device="cuda", dtype=torch.uint8)
    K.maxpool_fwd(a, p_ref, arg_ref)
    p = torch.empty_like(p_ref)
    arg = torch.empty_like(arg_ref)
    K.stem_bnrelu_maxpool(x, ms, g, b, p, arg)
    assert torch.equal(p, p_ref) and torch.equal(arg, arg_ref)
    dp = torch.randn(N, Hp, Hp, C, device="cuda").bfloat16()
    da = torch.empty_like(x)
    K.maxpool_bwd(dp, arg, da)
    red_ref = torch.zeros(C, 2, device="cuda")
    K.bn_bwd_reduce(da, a, x, ms, red_ref)
    dx_ref = torch.empty_like(x)
    dg_ref, db_ref = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    K.bn_bwd_apply(da, a, x, ms, g, red_ref, dx_ref, dg_ref, db_ref, training)
    red = torch.zeros(C, 2, device="cuda")
    dx = torch.empty_like(x)
    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
    K.stem_pool_bn_bwd(dp, arg, x, ms, g, b, red, dx, dg, db, training)
    assert torch.allclose(red, red_ref, rtol=1e-4, atol=1e-2)
    assert torch.allclose(dg, dg_ref, rtol=1e-4, atol=1e-2) and torch.allclose(db, db_ref, rtol=1e-4, atol=1e-2)
    assert rel_rms(dx.float(), dx_ref.float()) < 1e-2


def test_trunk_forward_backward_deterministic():
    """Every BatchNorm sum (forward statistics, fused and standalone backward reductions) is stored per row
    tile / block and folded in a fixed order -- no fp32 atomics anywhere in the trunk -- so a train-mode
    forward + backward is bitwise reproducible: features and every weight gradient."""
    from multimodalemotionrecognition_amd.video import trunk_backward, trunk_forward

    m, _ = build_trunk()
    m.train(True)
    video, _, _ = params.clip_inputs(1, frames=8, seed=43)
    x = torch.from_numpy(video[0]).cuda()
    outs, grads = [], []
    for _ in range(2):
        f, saved = trunk_forward(m, x, True)
        outs.append(f.clone())
        g = trunk_backward(m, saved, torch.ones_like(f), True)
        grads.append({k: v.clone() for k, v in g.items()})
        for q in m.parameters():
            q.grad = None
    assert torch.equal(outs[0], outs[1])
    for q in m.parameters():
        a, b = grads[0].get(id(q)), grads[1].get(id(q))
        if a is not None:
            assert torch.equal(a, b)


@pytest.mark.parametrize("transpose", [False, True])
def test_flat_pack_matches_2d_pack(transpose):
    """mer_pack_conv_weights_flat (the per-step re-pack: 1-D grid, column 8 = first block) == the 2-D-grid
    mer_pack_conv_weights bit for bit, for every ResNet18 conv (forward + s2d stem, or transposed)."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.video import ResNet18Trunk

    torch.manual_seed(7)
    trunk = ResNet18Trunk().cuda()
    trunk.pack_all(False)  # the transposed (mode 3) records read the forward packs
    plan = trunk._pack_plan(transpose)
    bufs = [plan["outs"][id(c)] for c in plan["convs"]]
    for b in bufs:
        b.fill_(1.0)
    K.pack_conv_weights(plan["desc"], plan["total"], flat=False)
    ref = [b.clone() for b in bufs]
    for b in bufs:
        b.fill_(-3.0)
    K.pack_conv_weights(plan["desc"], plan["blocks"])
    torch.cuda.synchronize()
    for c, b, r in zip(plan["convs"], bufs, ref):
        assert torch.equal(b, r), f"conv {tuple(c.weight.shape)} differs"


def test_transposed_pack_from_forward_pack():
    """Mode 3 (64x64 tile transpose of the forward bf16 pack, the per-step path) == mode 1 (the fp32 weights
    re-read and rounded) bit for bit for every non-stem ResNet18 conv, and == torch's own layout."""
    from multimodalemotionrecognition_amd import kernels as K
    from multimodalemotionrecognition_amd.video import ResNet18Trunk

    torch.manual_seed(11)
    trunk = ResNet18Trunk().cuda()
    trunk.pack_all(True)
    plan = trunk._pack_plan(True)
    assert all(int(m) == 3 for m in plan["desc"][:, 7].tolist())
    got = [plan["outs"][id(c)].clone() for c in plan["convs"]]
    rows, blocks = [], 0
    for c, r in zip(plan["convs"], plan["desc"].tolist()):
        Kc, C = r[2], r[3]
        rows.append([c.weight.data_ptr(), r[1], Kc, C, r[4], r[5], r[6], 1, blocks])
        blocks += r[6] * ((Kc + 63) // 64)
    K.pack_conv_weights(torch.tensor(rows, dtype=torch.int64).cuda(), blocks)
    torch.cuda.synchronize()
    for c, g in zip(plan["convs"], got):
        ref = plan["outs"][id(c)]
        assert torch.equal(g, ref), f"conv {tuple(c.weight.shape)} differs"
        Kc, C, R, S = c.weight.shape
        want = c.weight.detach().bfloat16().permute(1, 2, 3, 0).reshape(C, R * S * Kc)
        assert torch.equal(g, want)


@pytest.mark.parametrize("C,Kc,H", [(64, 128, 28), (128, 256, 14), (256, 512, 8)])
def test_dgrad_fused_downsample_vs_torch(C, Kc, H):
    """mer_conv_dgrad_ds: the 3x3/s2/p1 conv1 dgrad with the 1x1/s2 downsample's input gradient fused in as an extra
    K segment of parity class (0, 0) == torch's conv_transpose sum of the two branches on the same bf16 operands
    (one fp32 accumulator, one bf16 rounding), and within a bf16 rounding of the two-launch form."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(C)
    N = 2
    Ho = (H + 2 - 3) // 2 + 1
    dy = torch.randn(N, Kc, Ho, Ho).bfloat16().float()
    dyd = torch.randn(N, Kc, Ho, Ho).bfloat16().float()
    w = (torch.randn(Kc, C, 3, 3) / (9 * C) ** 0.5).bfloat16().float()
    wd = (torch.randn(Kc, C, 1, 1) / C ** 0.5).bfloat16().float()
    ref = F.conv_transpose2d(dy, w, stride=2, padding=1, output_padding=1) + \
        F.conv_transpose2d(dyd, wd, stride=2, output_padding=1)
    ref = ref[:, :, :H, :H]
    wt = w.permute(1, 2, 3, 0).reshape(C, 9 * Kc).contiguous().cuda().bfloat16()  # [C][r][s][k]
    wdt = wd.reshape(Kc, C).t().contiguous().cuda().bfloat16()                   # [C][k]
    dyh = dy.permute(0, 2, 3, 1).contiguous().cuda().bfloat16()
    dydh = dyd.permute(0, 2, 3, 1).contiguous().cuda().bfloat16()
    dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
    K.conv_dgrad(dyh, wt, dx, 3, 3, 2, 1, ds=(dydh, wdt))
    got = dx.float().permute(0, 3, 1, 2).cpu()
    assert rel_rms(got, ref) < 4e-3, rel_rms(got, ref)
    dxd = torch.empty_like(dx)
    K.conv_dgrad(dydh, wdt, dxd, 1, 1, 2, 0)
    dx2 = torch.empty_like(dx)
    K.conv_dgrad(dyh, wt, dx2, 3, 3, 2, 1, residual=dxd)
    assert rel_rms(got, dx2.float().permute(0, 3, 1, 2).cpu()) < 6e-3


@pytest.mark.parametrize("M,C", [(4096, 512), (4097, 512), (12544, 256), (50176, 128), (65536, 64), (200704, 64)])
def test_bn_finalize_and_partials_sum_all_row_counts(M, C):
    """mer_bn_finalize / mer_partials_sum over every row-count regime of the trunk at B = 32: <= 64 partial rows (one
    launch), 65..1024 rows (one 16-wave launch per 64 channels, round 6: layer2 / layer3), > 1024 rows (the two-stage
    fold: stem / layer1).  Against float64 sums of the same rows; running statistics as torch (momentum, unbiased
    variance); each launch bitwise repeatable."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(13)
    rows = K.bn_stat_rows(M)
    st = torch.zeros(rows, C, 2, device="cuda")
    data = rows - 64
    vals = torch.randn(data, C, 2, device="cuda")
    vals[..., 0] = vals[..., 0] * 3 + 1.0   # per-tile sums
    vals[..., 1] = vals[..., 1].abs() * 40 + 64.0  # per-tile sums of squares
    st[:data] = vals
    ref_sum = vals.double().sum(0).cpu()
    mean = ref_sum[:, 0] / M
    var = (ref_sum[:, 1] / M - mean * mean).clamp_min(0)
    outs = []
    for _ in range(2):
        ms = torch.empty(C, 2, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros((), dtype=torch.int64, device="cuda")
        K.bn_finalize(st.clone(), M, 1e-5, 0.1, ms, rm, rv, nbt)
        outs.append((ms, rm, rv, nbt))
    (ms, rm, rv, nbt), (ms2, rm2, rv2, _) = outs
    assert torch.equal(ms, ms2) and torch.equal(rm, rm2) and torch.equal(rv, rv2)
    assert torch.allclose(ms[:, 0].cpu().double(), mean, rtol=1e-5, atol=1e-6)
    assert torch.allclose(ms[:, 1].cpu().double(), (var + 1e-5).rsqrt(), rtol=1e-4)
    assert torch.allclose(rm.cpu().double(), 0.1 * mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(rv.cpu().double(), 0.9 + 0.1 * var * M / (M - 1), rtol=1e-4)
    assert int(nbt) == 1
    # the backward's partial-row fold: MER_BN_RED_ROWS(M) rows (+ the 64 scratch rows it may use)
    prow = K.bn_red_rows(M)
    parts = torch.zeros(prow, C, 2, device="cuda")
    parts[:prow - 64] = torch.randn(prow - 64, C, 2, device="cuda")
    s1 = K.partials_sum(parts.clone(), torch.empty(C, 2, device="cuda"))
    s2 = K.partials_sum(parts.clone(), torch.empty(C, 2, device="cuda"))
    assert torch.equal(s1, s2)
    ref = parts[:prow - 64].double().sum(0).cpu()
    assert torch.allclose(s1.cpu().double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("M,C", [(4096, 512), (12544, 256), (1000, 64)])
def test_bn_bwd_apply2_matches_two_launches(M, C):
    """mer_bn_bwd_apply2 (a stride-2 block's bn2 + downsample-BN backward applies over the shared gradient and ReLU
    mask, one launch) == two mer_bn_bwd_apply launches, bitwise, dgamma / dbeta accumulated (+=) the same way."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(23)
    bf = torch.bfloat16
    dy, mask, x, x2 = (torch.randn(M, C, device="cuda").to(bf) for _ in range(4))
    mss = [torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous() for _ in range(2)]
    gammas = [torch.randn(C, device="cuda") for _ in range(2)]
    reds = [torch.randn(C, 2, device="cuda") * 100 for _ in range(2)]
    for bs in (True, False):
        acc = [torch.randn(C, device="cuda") for _ in range(4)]
        ref = [a.clone() for a in acc]
        d1, d2 = torch.empty_like(x), torch.empty_like(x2)
        K.bn_bwd_apply(dy, mask, x, mss[0], gammas[0], reds[0], d1, ref[0], ref[1], bs)
        K.bn_bwd_apply(dy, mask, x2, mss[1], gammas[1], reds[1], d2, ref[2], ref[3], bs)
        e1, e2 = torch.empty_like(x), torch.empty_like(x2)
        K.bn_bwd_apply2(dy, mask, x, mss[0], gammas[0], reds[0], e1, acc[0], acc[1], x2, mss[1], gammas[1], reds[1],
                        e2, acc[2], acc[3], bs)
        assert torch.equal(d1, e1) and torch.equal(d2, e2), bs
        assert all(torch.equal(a, b) for a, b in zip(acc, ref)), bs


@pytest.mark.parametrize("M,C", [(4096, 512), (12544, 256), (50176, 128), (200704, 64)])
def test_bn_fold_pairs_match_single_launches(M, C):
    """mer_bn_finalize_rows2 / mer_partials_sum2 (a stride-2 block's bn2 + downsample-BN folds in one launch) against
    two single launches: bitwise where both take the wide kernel (65-1024 rows), to fp32 rounding where a single call
    takes the <= 64-row or two-stage form; running statistics and num_batches_tracked updated per record."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(29)
    rows = K.bn_stat_rows(M)
    data = rows - 64
    recs = []
    for _ in range(2):
        st = torch.zeros(rows, C, 2, device="cuda")
        st[:data, :, 0] = torch.randn(data, C, device="cuda") * 3 + 1.0
        st[:data, :, 1] = torch.randn(data, C, device="cuda").abs() * 40 + 64.0
        recs.append(st)
    exact = 64 < data <= 1024
    single, paired = [], []
    for st in recs:
        ms, rm, rv = torch.empty(C, 2, device="cuda"), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros((), dtype=torch.int64, device="cuda")
        K.bn_finalize(st.clone(), M, 1e-5, 0.1, ms, rm, rv, nbt)
        single.append((ms, rm, rv, nbt))
    args = []
    for st in recs:
        ms, rm, rv = torch.empty(C, 2, device="cuda"), torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros((), dtype=torch.int64, device="cuda")
        args.append((st.clone(), M, ms, rm, rv, nbt, None))
        paired.append((ms, rm, rv, nbt))
    K.bn_finalize_pair(args[0], args[1], 1e-5, 0.1)
    for a, b in zip(single, paired):
        for x, y in zip(a, b):
            assert torch.equal(x, y) if exact or x.dtype == torch.int64 else torch.allclose(x, y, rtol=2e-6, atol=1e-6)
    prow = K.bn_red_rows(M)
    bufs = [torch.randn(prow, C, 2, device="cuda") for _ in range(2)]
    for b in bufs:
        b[prow - 64:] = 0
    s = [K.partials_sum(b.clone(), torch.empty(C, 2, device="cuda")) for b in bufs]
    p = K.partials_sum_pair(bufs[0].clone(), torch.empty(C, 2, device="cuda"), bufs[1].clone(),
                            torch.empty(C, 2, device="cuda"))
    pexact = 64 < prow - 64 <= 1024
    for x, y in zip(s, p):
        assert torch.equal(x, y) if pexact else torch.allclose(x, y, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape", [(256, 28, 64, 64, 3, 1), (256, 28, 64, 128, 3, 2), (256, 14, 128, 128, 3, 1),
                                   (256, 28, 64, 128, 1, 2), (256, 14, 128, 256, 3, 2), (256, 7, 256, 256, 3, 1),
                                   (256, 7, 256, 512, 3, 2), (256, 4, 512, 512, 3, 1), (40, 14, 128, 128, 3, 1)])
def test_conv_fwd_rows_exact_for_default_variant(shape):
    """With the default variant, K.conv_fwd's returned row count is exact: every statistics row below it is written
    (the trunk's forward arena is therefore not zeroed), and the finalize over those rows of a NaN-filled buffer equals
    the finalize of a zeroed one.  The ResNet18 forward convs at B = 32 (and a small batch)."""
    from multimodalemotionrecognition_amd import kernels as K

    N, H, C, Kc, R, s = shape
    pad = R // 2
    torch.manual_seed(31)
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = torch.randn(Kc, C, R, R, device="cuda") / (R * (C ** 0.5))
    wp = torch.empty(Kc, R * R * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    Ho = (H + 2 * pad - R) // s + 1
    M = N * Ho * Ho
    outs = []
    for fill in (0.0, float("nan")):
        y = torch.empty(N, Ho, Ho, Kc, device="cuda", dtype=torch.bfloat16)
        st = torch.full((K.bn_stat_rows(M), Kc, 2), fill, device="cuda")
        rows = K.conv_fwd(x, wp, y, st, R, R, s, pad)
        assert not torch.isnan(st[:rows]).any(), rows
        ms = torch.empty(Kc, 2, device="cuda")
        K.bn_finalize(st, M, 1e-5, 0.1, ms, rows=rows)
        outs.append(ms)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("shape", [(256, 28, 64, 64, 1, False, False), (256, 28, 64, 128, 2, True, False),
                                   (256, 14, 128, 128, 1, False, True), (256, 14, 128, 256, 2, True, False),
                                   (256, 7, 256, 256, 1, False, True), (256, 7, 256, 512, 2, True, False),
                                   (256, 4, 512, 512, 1, False, False), (40, 14, 128, 128, 1, False, False),
                                   (40, 14, 128, 256, 2, False, False)])
def test_conv_dgrad_rows_exact_for_default_variant(shape):
    """With the default variant, K.conv_dgrad's returned reduction row count is exact for the stride-1 and the
    parity-class stride-2 dgrads (with the fused downsample segment and with a second BN): every row below it is
    written (the trunk backward's reduction arena is not zeroed), and the fold over those rows of a NaN-filled buffer
    equals the fold of a zeroed one.  The ResNet18 input gradients at B = 32 (and a small batch)."""
    from multimodalemotionrecognition_amd import kernels as K

    N, H, C, Kc, s, ds, two = shape  # dx [N, H, H, C] <- dy [N, H/s, H/s, Kc]
    torch.manual_seed(37)
    Ho = (H + 2 - 3) // s + 1
    dy = torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16()
    w = torch.randn(Kc, C, 3, 3, device="cuda") / (3 * Kc ** 0.5)
    wt = torch.empty(C, 9 * Kc, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wt, C, True)
    kw = {}
    if ds:
        wd = torch.randn(Kc, C, 1, 1, device="cuda") / Kc ** 0.5
        wdt = torch.empty(C, Kc, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(wd, wdt, C, True)
        kw["ds"] = (torch.randn(N, Ho, Ho, Kc, device="cuda").bfloat16(), wdt)
    mask, xb, xb2 = (torch.randn(N, H, H, C, device="cuda").bfloat16() for _ in range(3))
    ms = torch.stack([torch.randn(C), torch.rand(C) + 0.5], 1).cuda().contiguous()
    M = N * H * H
    res = []
    for fill in (0.0, float("nan")):
        reds = [torch.full((K.bn_red_rows(M), C, 2), fill, device="cuda") for _ in range(2)]
        bnr = (mask, xb, ms, reds[0]) + ((xb2, ms, reds[1]) if two else ())
        dx = torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16)
        rows = K.conv_dgrad(dy, wt, dx, 3, 3, s, 1, bnr=bnr, **kw)
        out = []
        for red in reds[:2 if two else 1]:
            assert not torch.isnan(red[:rows]).any(), rows
            out.append(K.partials_sum(red, torch.empty(C, 2, device="cuda"), rows))
        res.append(out)
    for a, b in zip(*res):
        assert torch.equal(a, b)
