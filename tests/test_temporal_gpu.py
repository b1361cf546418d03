"""TemporalPooler 'attn' / 'transformer' on the HIP schedule (temporal_hip.py) -- SURVEY §8(f) rank 2.

* Pinned against the reference itself: ``temporal_{attn,transformer}.npz`` (TemporalPooler(dim=8,
  heads=2) imported from the reference, tools/gen_golden.py) and ``xattn_small_{attn,transformer}.npz``
  (FusionModel xattn with those poolers at the reference tests' d_model=8 / heads=2 shapes).
* Gradients at the north-star head shapes (d_model=128, T=8, Ta=149) against the fp32 oracle's autograd
  (oracle/fusion_ref.py, itself pinned by the goldens above).  Tolerances: logits 1e-4, gradients 2e-4
  relative to each tensor's max.
"""
import pytest
import torch

from oracle import fusion_ref, params
from tests.gpu_helpers import feats, head_model, max_abs
from tests.helpers import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["mean", "attn", "transformer"])
def test_temporal_pooler_vs_reference_golden(mode):
    from multimodalemotionrecognition_amd.temporal import TemporalPooler

    g = golden(f"temporal_{mode}.npz")
    pool = TemporalPooler(dim=8, mode=mode, num_heads=2, num_layers=1, dropout=0.0)
    sd = pool.state_dict()
    assert sorted(sd) == sorted(str(n) for n in g["names"])
    pool.load_state_dict({k: torch.from_numpy(params.init_tensor(k, tuple(v.shape), 0)) for k, v in sd.items()})
    pool = pool.cuda().eval()
    with torch.no_grad():
        y = pool(torch.from_numpy(g["x"]).cuda())
    assert max_abs(y, g["y"]) < 1e-5


@pytest.mark.parametrize("pooling", ["attn", "transformer"])
def test_xattn_small_shapes_with_pooling(pooling):
    """d_model=8, num_heads=2 as in the reference's test_attention_integration.py:102-125."""
    g = golden(f"xattn_small_{pooling}.npz")
    m = head_model("concat", False, d_model=8, heads=2, v_dim=16, seq_dim=8, pooling=pooling, t_heads=2,
                   t_dropout=0.0).eval()
    v, a = feats(2, 4, 12, v_dim=16, a_dim=8, seed=11)
    with torch.no_grad():
        logits = m(v[..., None, None], a)
    assert tuple(logits.shape) == (2, 8)
    assert max_abs(logits, g["logits"]) < 1e-4


@pytest.mark.parametrize("pooling", ["attn", "transformer"])
def test_xattn_pooling_grads_vs_oracle(pooling):
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss

    m = head_model("concat", False, pooling=pooling, t_dropout=0.0).eval()
    v, a = feats(4, 8, 149, seed=3)
    v.requires_grad_(True)
    labels = torch.tensor([0, 3, 7, 2]).cuda()
    loss = CrossEntropyLoss(label_smoothing=0.1)(m.xattn_from_features(v, a), labels)
    loss.backward()
    p = {k: torch.from_numpy(x) for k, x in params.init_state(
        fusion_ref.xattn_head_param_shapes(temporal_pooling=pooling)).items()}
    for q in p.values():
        q.requires_grad_(True)
    vr = v.detach().cpu().requires_grad_(True)
    ref, _ = fusion_ref.xattn_forward(p, vr, a.cpu(), temporal_pooling=pooling)
    rl = fusion_ref.cross_entropy(ref, labels.cpu(), label_smoothing=0.1)
    rl.backward()
    assert abs(float(loss.detach()) - float(rl.detach())) < 1e-5
    assert max_abs(v.grad, vr.grad) / max(1e-6, float(vr.grad.abs().max())) < 2e-4
    checked = 0
    for n, q in m.named_parameters():
        if n.startswith(("audio_model", "video_model", "audio_time_conv")):
            continue
        r = p[n].grad
        assert q.grad is not None, n
        # score.4.bias: softmax is shift-invariant, its exact gradient is 0 (fp32 noise ~1e-8 on both sides)
        scale = max(1e-2, float(r.abs().max()))
        assert max_abs(q.grad, r) / scale < 2e-4, n
        checked += 1
    assert checked > (20 if pooling == "attn" else 40)


def test_transformer_pooler_long_sequence_backward():
    """Self-attention over Ta=149 exceeds the fused MHA backward's LDS image: the materialised per-head
    path (batched f32 GEMMs + mer_softmax_dropout_bwd) must give the oracle's gradients."""
    from multimodalemotionrecognition_amd.temporal import TemporalPooler

    pool = TemporalPooler(dim=128, mode="transformer", num_heads=4, num_layers=1, dropout=0.0)
    sd = pool.state_dict()
    pool.load_state_dict({k: torch.from_numpy(params.init_tensor(k, tuple(v.shape), 0)) for k, v in sd.items()})
    pool = pool.cuda().eval()
    torch.manual_seed(0)
    x = torch.randn(3, 149, 128)
    xd = x.cuda().requires_grad_(True)
    y = pool(xd)
    w = torch.randn(3, 128)
    (y * w.cuda()).sum().backward()
    p = {"p." + k: v.detach().cpu().clone().requires_grad_(True) for k, v in pool.named_parameters()}
    xr = x.clone().requires_grad_(True)
    yr = fusion_ref.temporal_pool(xr, p, "p", "transformer", 4, 1)
    (yr * w).sum().backward()
    assert max_abs(y, yr) < 1e-4
    assert max_abs(xd.grad, xr.grad) / float(xr.grad.abs().max()) < 2e-4
    for n, q in pool.named_parameters():
        r = p["p." + n].grad
        assert max_abs(q.grad, r) / max(1e-2, float(r.abs().max())) < 2e-4, n


def test_pooling_dropout_reproducible_in_train_mode():
    m = head_model("concat", False, pooling="transformer").train()
    v, a = feats(4, 8, 149, seed=5)
    torch.manual_seed(0)
    l1 = m.xattn_from_features(v, a)
    torch.manual_seed(0)
    l2 = m.xattn_from_features(v, a)
    torch.manual_seed(1)
    l3 = m.xattn_from_features(v, a)
    assert torch.equal(l1, l2) and not torch.equal(l1, l3)
    assert torch.isfinite(l1).all()
