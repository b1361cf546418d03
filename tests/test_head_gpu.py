"""GPU parity of the fp32 fusion-head kernels against the oracle / reference goldens.

Tolerance (north star): logits within 1e-3 of the CPU reference; the fp32 MFMA path is
expected ~1e-5, so the tests assert 1e-4 on logits and explicit bounds on gradients.
"""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, params
from tests.gpu_helpers import feats, head_model, max_abs, oracle_head_params
from tests.helpers import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("head", ["concat", "gated"])
@pytest.mark.parametrize("prior", [0, 1])
def test_xattn_c1_logits_vs_reference_golden(head, prior):
    g = golden(f"xattn_c1_{head}_prior{prior}.npz")
    m = head_model(head, bool(prior)).eval()
    v, a = feats(2, 8, 64)
    with torch.no_grad():
        logits = m(v[..., None, None], a)  # full FusionModel.forward with identity encoders (ref test pattern)
    assert tuple(logits.shape) == (2, 8)
    assert max_abs(logits, g["logits"]) < 1e-4


@pytest.mark.parametrize("head,prior", [("concat", 0), ("concat", 1), ("gated", 0)])
def test_xattn_c2_logits(head, prior):
    g = golden(f"xattn_c2_{head}_prior{prior}.npz")
    m = head_model(head, bool(prior)).eval()
    v, a = feats(32, 8, 149, seed=7)
    with torch.no_grad():
        logits = m.xattn_from_features(v, a)
    assert max_abs(logits, g["logits"]) < 1e-4


def test_xattn_c2_grads_and_fused_adam():
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss
    from multimodalemotionrecognition_amd.optim import FusedAdam

    g = golden("xattn_c2_concat_prior0.npz")
    m = head_model("concat", False).eval()
    v, a = feats(32, 8, 149, seed=7)
    v.requires_grad_(True)
    labels = torch.from_numpy(g["labels"]).cuda()
    trainable = [(n, q) for n, q in m.named_parameters() if not n.startswith(("audio_model", "video_model"))]
    opt = FusedAdam([q for _, q in trainable], lr=1e-3, weight_decay=1e-4)
    opt.zero_grad()
    logits = m.xattn_from_features(v, a)
    loss = CrossEntropyLoss()(logits, labels)
    loss.backward()
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-5
    assert max_abs(v.grad[:2], g["grad_v"]) < 1e-6
    for n, q in trainable:
        key = "grad." + n
        if key in g.files:
            ref = g[key]
            scale = max(1e-3, float(np.abs(ref).max()))
            assert max_abs(q.grad, ref) / scale < 1e-4, n
        else:
            assert q.grad is None, f"{n} must receive no gradient (dead on the WavLM path)"
    # Adam's first step is ~lr*sign(g): feed the reference's own gradients so the optimizer
    # kernel is checked exactly, independent of 1e-9 gradient noise on |g|~eps elements.
    with torch.no_grad():
        for n, q in trainable:
            if "grad." + n in g.files:
                q.grad.copy_(torch.from_numpy(g["grad." + n]))
    opt.step()
    for n, q in trainable:
        key = "adam1." + n
        if key in g.files:
            assert max_abs(q, g[key]) < 2e-6, n


@pytest.mark.parametrize("head", ["concat", "gated"])
def test_xattn_prior_grads_vs_oracle(head):
    """Prior-bias path gradients (no reference grad golden for it): oracle autograd is the checker."""
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss

    m = head_model(head, True).eval()
    v, a = feats(4, 8, 149, seed=3)
    labels = torch.tensor([0, 3, 7, 2]).cuda()
    loss = CrossEntropyLoss(label_smoothing=0.1)(m.xattn_from_features(v, a), labels)
    loss.backward()
    p = oracle_head_params(head, True)
    for q in p.values():
        q.requires_grad_(True)
    ref, _ = fusion_ref.xattn_forward(p, v.cpu(), a.cpu(), xattn_head=head, use_prior=True)
    rl = fusion_ref.cross_entropy(ref, labels.cpu(), label_smoothing=0.1)
    rl.backward()
    assert abs(float(loss.detach()) - float(rl.detach())) < 1e-5
    for n, q in m.named_parameters():
        if n.startswith(("audio_model", "video_model")) or n.startswith("audio_time_conv"):
            continue
        r = p[n].grad
        assert q.grad is not None, n
        scale = max(1e-4, float(r.abs().max()))
        assert max_abs(q.grad, r) / scale < 2e-4, n


@pytest.mark.parametrize("pooling", ["mean"])
def test_reference_test_shapes(pooling):
    """d_model=8, num_heads=2 as in the reference's test_attention_integration.py:80-100."""
    g = golden(f"xattn_small_{pooling}.npz")
    m = head_model("concat", False, d_model=8, heads=2, v_dim=16, seq_dim=8).eval()
    v, a = feats(2, 4, 12, v_dim=16, a_dim=8, seed=11)
    with torch.no_grad():
        logits = m(v[..., None, None], a)
    assert tuple(logits.shape) == (2, 8)
    assert max_abs(logits, g["logits"]) < 1e-4


def test_train_mode_dropout_statistics():
    """MHA dropout / drop-path / MLP dropout cannot bit-match torch's RNG: check keep-rate & scaling."""
    from multimodalemotionrecognition_amd import kernels as K

    x = torch.ones(1000, 1000, device="cuda")
    K.dropout_(x, 0.2, torch.full((1,), 1234, dtype=torch.int64, device="cuda"), 3)
    kept = (x != 0).float().mean().item()
    assert abs(kept - 0.8) < 0.005
    assert torch.allclose(x[x != 0], torch.full_like(x[x != 0], 1 / 0.8))
    m = head_model("concat", False).train()
    v, a = feats(8, 8, 149, seed=5)
    torch.manual_seed(0)
    l1 = m.xattn_from_features(v, a)
    torch.manual_seed(0)
    l2 = m.xattn_from_features(v, a)
    torch.manual_seed(1)
    l3 = m.xattn_from_features(v, a)
    assert torch.equal(l1, l2), "same host seed must reproduce the same masks"
    assert not torch.equal(l1, l3)
    assert torch.isfinite(l1).all()


def test_gemm_f32_transposes():
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(0)
    for (M, N, Kd) in [(1, 1, 1), (5, 7, 3), (64, 64, 16), (130, 70, 300), (4768, 128, 768)]:
        a = torch.randn(M, Kd)
        b = torch.randn(Kd, N)
        ref = a @ b
        for ta in (False, True):
            for tb in (False, True):
                ad = (a.t().contiguous() if ta else a).cuda()
                bd = (b.t().contiguous() if tb else b).cuda()
                out = torch.empty(M, N, device="cuda")
                K.gemm(ad, bd, out, trans_a=ta, trans_b=tb)
                assert max_abs(out, ref) < 1e-3 * max(1.0, Kd ** 0.5), (M, N, Kd, ta, tb)
    # bf16 operands (16-byte segment loads) and unaligned views (scalar segment path)
    for (M, N, Kd) in [(37, 45, 70), (4768, 128, 768), (256, 512, 128)]:
        a = torch.randn(M, Kd).bfloat16().float()
        b = torch.randn(Kd, N).bfloat16().float()
        ref = a @ b
        for adt, bdt in ((torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16)):
            for tb in (False, True):
                bd = (b.t().contiguous() if tb else b).to(bdt).cuda()
                out = torch.empty(M, N, device="cuda")
                K.gemm(a.to(adt).cuda(), bd, out, trans_b=tb)
                assert max_abs(out, ref) < 1e-3 * max(1.0, Kd ** 0.5), (M, N, Kd, adt, bdt, tb)
        big = torch.randn(M, Kd + 1)
        big[:, 1:] = a
        out = torch.empty(M, N, device="cuda")
        K.gemm(big.cuda()[:, 1:], b.cuda(), out)
        assert max_abs(out, ref) < 1e-3 * max(1.0, Kd ** 0.5), (M, N, Kd, "unaligned")
    # split-K accumulate path
    a = torch.randn(4768, 128)
    x = torch.randn(4768, 768)
    out = torch.zeros(128, 768, device="cuda")
    K.gemm(a.cuda(), x.cuda(), out, trans_a=True, beta=1, splitk=8)
    assert max_abs(out, a.t() @ x) < 5e-3
    # the K slices are summed in slice order (no atomics): bitwise reproducible
    out2 = torch.zeros(128, 768, device="cuda")
    K.gemm(a.cuda(), x.cuda(), out2, trans_a=True, beta=1, splitk=8)
    assert torch.equal(out, out2)


def test_late_and_ce_kernels():
    from multimodalemotionrecognition_amd.embedding_head import late_probs
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss, LateNLLLoss

    torch.manual_seed(0)
    za, zv = torch.randn(6, 8), torch.randn(6, 8)
    y = torch.randint(0, 8, (6,))
    zad, zvd = za.cuda().requires_grad_(True), zv.cuda().requires_grad_(True)
    pr = late_probs(zad, zvd)
    loss = LateNLLLoss()(pr, y.cuda())
    loss.backward()
    za.requires_grad_(True)
    zv.requires_grad_(True)
    rp = fusion_ref.late_forward(za, zv)
    rl = fusion_ref.late_nll(rp, y)
    rl.backward()
    assert max_abs(pr, rp) < 1e-6
    assert abs(float(loss.detach()) - float(rl.detach())) < 1e-5
    assert max_abs(zad.grad, za.grad) < 1e-6
    z = torch.randn(5, 8, requires_grad=True)
    zd = z.detach().cuda().requires_grad_(True)
    y = torch.randint(0, 8, (5,))
    l1 = CrossEntropyLoss(0.1)(zd, y.cuda()) * 3.0
    l1.backward()
    l2 = torch.nn.functional.cross_entropy(z, y, label_smoothing=0.1) * 3.0
    l2.backward()
    assert abs(float(l1.detach()) - float(l2.detach())) < 1e-5
    assert max_abs(zd.grad, z.grad) < 1e-6


@pytest.mark.parametrize("B,C", [(1, 8), (32, 8), (100, 8), (33, 3), (40, 13), (7, 64), (9, 70)])
def test_ce_kernel_shapes_and_top1(B, C):
    """ce_kernel<G> (one lane group per row, several passes when B > 256 / G, a lane looping over classes when
    C > 64): loss, logits gradient and top-1 vs torch (label smoothing 0.1), ties resolved to the lowest index."""
    from multimodalemotionrecognition_amd import kernels as K

    g = torch.Generator().manual_seed(B * 100 + C)
    z = torch.randn(B, C, generator=g)
    z[0, : min(C, 3)] = 2.5  # a tie for the top-1
    y = torch.randint(0, C, (B,), generator=g)
    loss = torch.empty((), device="cuda")
    dl = torch.empty(B, C, device="cuda")
    pred = torch.empty(B, dtype=torch.int64, device="cuda")
    K.cross_entropy(z.cuda(), y.cuda(), loss, dl, label_smoothing=0.1, preds=pred)
    zr = z.clone().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(zr, y, label_smoothing=0.1)
    lr.backward()
    assert abs(float(loss) - float(lr)) < 1e-5 * max(1.0, float(lr))
    assert max_abs(dl, zr.grad) < 1e-6
    assert torch.equal(pred.cpu(), z.argmax(dim=1))


@pytest.mark.parametrize("mode", ["concat", "gated", "late"])
def test_c4_embedding_heads(mode):
    """late / concat / gated heads at feature level vs the reference goldens (fusion.py:358-363,413-435)."""
    from multimodalemotionrecognition_amd.embedding_head import late_probs
    from multimodalemotionrecognition_amd.fusion import FusionModel

    g = golden(f"c4_{mode}.npz")

    class Enc(torch.nn.Module):
        def __init__(self, dim):
            super().__init__()
            self.embedding_dim = dim

        def encode(self, x):
            return x

    m = FusionModel(Enc(768), Enc(512), num_classes=8, mode=mode)
    names = [str(n) for n in g["names"]]
    if mode == "late":
        sd = {n: torch.from_numpy(params.init_tensor(n, s)) for n, s in
              [("audio_model.classifier.0.weight", (768, 768)), ("audio_model.classifier.0.bias", (768,)),
               ("audio_model.classifier.3.weight", (8, 768)), ("audio_model.classifier.3.bias", (8,)),
               ("video_model.classifier.weight", (8, 512)), ("video_model.classifier.bias", (8,))]}
        a, v = torch.from_numpy(g["a_emb"]), torch.from_numpy(g["v_emb"])
        al = fusion_ref.linear(torch.relu(fusion_ref.linear(a, sd, "audio_model.classifier.0")), sd,
                               "audio_model.classifier.3")
        vl = fusion_ref.linear(v, sd, "video_model.classifier")
        out = late_probs(al.cuda(), vl.cuda())
    else:
        sd = m.state_dict()
        new = {k: torch.from_numpy(params.init_tensor(k, tuple(t.shape))) for k, t in sd.items()}
        if mode == "gated":
            new["gate.0.bias"].fill_(-1.0)
            new["gate.3.bias"].fill_(-1.0)
        assert sorted(k for k in names if not k.startswith(("audio_model", "video_model"))) == sorted(new)
        m.load_state_dict(new)
        m = m.cuda().eval()
        with torch.no_grad():
            out = m(torch.from_numpy(g["v_emb"]).cuda(), torch.from_numpy(g["a_emb"]).cuda())
    assert max_abs(out, g["out"]) < 1e-4


def test_colsum_and_layernorm_paths():
    """colsum (bias grads) and the row LayerNorm on its 4-wide (d % 256 == 0) and scalar paths."""
    from multimodalemotionrecognition_amd import kernels as K

    torch.manual_seed(3)
    for M, N in [(1, 3), (4768, 128), (300, 768), (17, 1000)]:
        x = torch.randn(M, N)
        out = torch.zeros(N, device="cuda")
        K.colsum(x.cuda(), out)
        assert max_abs(out, x.sum(0)) < 1e-3 * max(1.0, M ** 0.5)
        out2 = torch.zeros(N, device="cuda")
        K.colsum(x.cuda(), out2)
        assert torch.equal(out, out2), (M, N)  # fixed-order block fold
    for rows, d in [(4768, 768), (5, 512), (33, 200), (7, 1024)]:
        x = torch.randn(rows, d) * 3 + 1
        g, b = torch.randn(d), torch.randn(d)
        ref = torch.nn.functional.layer_norm(x, (d,), g, b, 1e-5)
        for idt, odt in ((torch.float32, torch.bfloat16), (torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                         (torch.bfloat16, torch.float32)):
            xi = x.to(idt)
            r = torch.nn.functional.layer_norm(xi.float(), (d,), g, b, 1e-5)
            y = torch.empty(rows, d, device="cuda", dtype=odt)
            K.layernorm(xi.cuda(), g.cuda(), b.cuda(), y)
            tol = 2e-4 if odt == torch.float32 else 2e-2 * float(r.abs().max())
            assert max_abs(y.float(), r) < tol, (rows, d, idt, odt)
