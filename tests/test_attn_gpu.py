"""GPU parity of the f32-MFMA multi-head attention core (attn.hip: mer_mha_fwd / mer_mha_bwd) against a
plain torch fp32 restatement of nn.MultiheadAttention's explicit path (TORCH:6576-6606) with the
per-sample additive bias of the emotion prior (fusion.py:351-354).  Shapes: the xattn blocks at the
north-star config (v2a Lq=8/Lk=149, a2v Lq=149/Lk=8, dh=32), the reference tests' d_model=8/heads=2
(dh=4), the temporal transformer pooler's self-attention, and ragged edges (Lq, Lk not multiples of 16).
Tolerance: fp32 throughout, 2e-5 absolute on O, 1e-4 relative on the gradients."""
import math

import pytest
import torch

from multimodalemotionrecognition_amd import kernels as K

pytestmark = pytest.mark.gpu

SHAPES = [  # B, H, Lq, Lk, dh
    (32, 4, 8, 149, 32),
    (32, 4, 149, 8, 32),
    (2, 2, 4, 12, 4),
    (2, 2, 12, 4, 4),
    (3, 4, 8, 8, 32),
    (2, 1, 17, 33, 64),
    (1, 3, 1, 1, 8),
    (5, 2, 40, 256, 16),
]


def _ref(q, k, v, bias, B, H, Lq, Lk, dh):
    qh = q.view(B, Lq, H, dh).transpose(1, 2)
    kh = k.view(B, Lk, H, dh).transpose(1, 2)
    vh = v.view(B, Lk, H, dh).transpose(1, 2)
    s = (qh * math.sqrt(1.0 / dh)) @ kh.transpose(-1, -2)
    if bias is not None:
        s = s + bias[:, None]
    p = torch.softmax(s, dim=-1)
    return (p @ vh).transpose(1, 2).reshape(B * Lq, H * dh), p


@pytest.mark.parametrize("B,H,Lq,Lk,dh", SHAPES)
@pytest.mark.parametrize("with_bias", [False, True])
def test_mha_fwd_bwd_vs_torch(B, H, Lq, Lk, dh, with_bias):
    g = torch.Generator().manual_seed(B * 1000 + Lq * 10 + Lk)
    d = H * dh
    # q in a wider row (ld != d) like the fused QKV projections of the head
    qbuf = torch.randn(B * Lq, d + 8, generator=g)
    kv = torch.randn(B * Lk, 2 * d, generator=g)
    bias = torch.randn(B, Lq, Lk, generator=g) if with_bias else None
    dO = torch.randn(B * Lq, d, generator=g)
    q, k, v = qbuf[:, :d], kv[:, :d], kv[:, d:]

    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    br = bias.clone().requires_grad_(True) if with_bias else None
    o_ref, p_ref = _ref(qr, kr, vr, br, B, H, Lq, Lk, dh)
    (o_ref * dO).sum().backward()

    qd, kvd, dOd = qbuf.cuda(), kv.cuda(), dO.cuda()
    bd = bias.cuda() if with_bias else None
    o = torch.empty(B * Lq, d, device="cuda")
    P = torch.empty(B, H, Lq, Lk, device="cuda")
    K.mha_fwd(qd[:, :d], kvd[:, :d], kvd[:, d:], bd, o, P, B, H, Lq, Lk)
    assert float((o.cpu() - o_ref.detach()).abs().max()) < 2e-5
    assert float((P.cpu() - p_ref.detach()).abs().max()) < 2e-6

    dq = torch.empty(B * Lq, d, device="cuda")
    dkv = torch.empty(B * Lk, 2 * d, device="cuda")
    db = torch.empty(B, Lq, Lk, device="cuda") if with_bias else None
    K.mha_bwd(qd[:, :d], kvd[:, :d], kvd[:, d:], P, dOd, dq, dkv[:, :d], dkv[:, d:], db, B, H, Lq, Lk)
    for got, ref in ((dq, qr.grad), (dkv[:, :d], kr.grad), (dkv[:, d:], vr.grad)) + (((db, br.grad),) if with_bias else ()):
        scale = max(1e-3, float(ref.abs().max()))
        assert float((got.cpu() - ref).abs().max()) / scale < 1e-4


def test_mha_dropout_mask_regenerated_in_backward():
    """Train mode: keep-rate and 1/(1-p) scaling of the attention dropout, and backward == the product
    rule applied with the SAME mask (dropped probabilities contribute no gradient to V)."""
    B, H, Lq, Lk, dh, p = 4, 4, 149, 8, 32, 0.3
    d = H * dh
    torch.manual_seed(0)
    q = torch.randn(B * Lq, d, device="cuda")
    kv = torch.randn(B * Lk, 2 * d, device="cuda")
    rng = torch.full((1,), 99, dtype=torch.int64, device="cuda")
    o0 = torch.empty(B * Lq, d, device="cuda")
    o1 = torch.empty(B * Lq, d, device="cuda")
    P = torch.empty(B, H, Lq, Lk, device="cuda")
    K.mha_fwd(q, kv[:, :d], kv[:, d:], None, o0, P, B, H, Lq, Lk, drop_p=p, rng=rng, site=7)
    K.mha_fwd(q, kv[:, :d], kv[:, d:], None, o1, P, B, H, Lq, Lk, drop_p=p, rng=rng, site=7)
    assert torch.equal(o0, o1)
    # dV = P'^T dO with dO = one-hot on one output column recovers column sums of P' per head
    dO = torch.zeros(B * Lq, d, device="cuda")
    dO[:, 0] = 1.0  # head 0, channel 0
    dq = torch.empty(B * Lq, d, device="cuda")
    dkv = torch.empty(B * Lk, 2 * d, device="cuda")
    K.mha_bwd(q, kv[:, :d], kv[:, d:], P, dO, dq, dkv[:, :d], dkv[:, d:], None, B, H, Lq, Lk, drop_p=p, rng=rng, site=7)
    colsum_pd = dkv[:, d].view(B, Lk)  # sum_i P'[b,0,i,j]
    colsum_p = P[:, 0].sum(1)
    ratio = (colsum_pd / colsum_p).mean().item()
    assert abs(ratio - 1.0) < 0.1  # E[m] = 1
    nz = (dkv[:, d] != 0).float().mean().item()
    assert nz > 0.99
