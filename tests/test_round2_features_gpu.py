"""GPU parity of the SURVEY 8(a.15) / 8(f) pieces added in round 2, against the imported-reference goldens:

* fusion_align_mode="clip" (ClipStyleAlignment, fusion.py:127-150, 417-418; loss combination train.py:221-225);
* dynamic INT8 with the emotion-prior adapter (optimized_runtime.py:95-96 quantizes prior_net and the four
  token-bias Linears too);
* TemporalPooler('transformer') at the encoders' widths (head_dim 128 / 192, train.py:357-443);
* gated-mode ModalityDropout gradient semantics (fusion.py:47-53, 430: the dropped projection and encoder
  get NO gradient, so torch Adam leaves them untouched).
"""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, int8_ref, params
from tests.gpu_helpers import feats, head_model, max_abs
from tests.helpers import check_grad, clip_head_params, golden, xattn_params

pytestmark = pytest.mark.gpu


class _Enc(torch.nn.Module):
    """Feature-level encoder stub (the reference tests' pattern): encode = identity."""

    def __init__(self, dim):
        super().__init__()
        self.embedding_dim = dim
        self.sequence_dim = dim

    def encode(self, x):
        return x


def _clip_model(mode):
    from multimodalemotionrecognition_amd.fusion import FusionModel

    m = FusionModel(_Enc(768), _Enc(512), num_classes=8, mode=mode, fusion_align_mode="clip", fusion_align_dim=256,
                    fusion_align_temperature=0.07)
    p = clip_head_params(mode)
    assert sorted(m.state_dict()) == sorted(p)
    m.load_state_dict(p)
    return m.cuda()


@pytest.mark.parametrize("mode", ["concat", "gated"])
def test_clip_alignment_vs_reference_golden(mode):
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss, add_scaled

    g = golden(f"c4_clip_{mode}.npz")
    m = _clip_model(mode).eval()
    a = torch.from_numpy(g["a_emb"]).cuda().requires_grad_(True)
    v = torch.from_numpy(g["v_emb"]).cuda().requires_grad_(True)
    logits = m(v, a)
    align = m.pop_alignment_loss()
    assert m.pop_alignment_loss() is None  # popped once (fusion.py:346-349)
    loss = add_scaled(CrossEntropyLoss()(logits, torch.from_numpy(g["labels"]).cuda()), align, 0.5)
    loss.backward()
    assert max_abs(logits, g["logits"]) < 1e-4
    assert abs(float(align.detach()) - float(g["align"])) < 1e-5
    assert abs(float(loss.detach()) - float(g["loss"])) < 1e-5
    assert max_abs(a.grad, g["grad_a"]) < 1e-5 * max(1.0, float(np.abs(g["grad_a"]).max()))
    assert max_abs(v.grad, g["grad_v"]) < 1e-5 * max(1.0, float(np.abs(g["grad_v"]).max()))
    for n, q in m.named_parameters():
        check_grad(g, n, q.grad.cpu(), atol=1e-5)


def test_clip_alignment_train_step_loss_combination():
    """TrainStep(fusion_align_weight=w): loss = cls + w * align (train.py:221-225); cls / contrastive reported."""
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, make_loss

    g = golden("c4_clip_concat.npz")
    m = _clip_model("concat").train()
    m.fusion[2].p = 0.0
    opt = build_optimizer(m)
    step = TrainStep(m, opt, make_loss("concat"), "concat", fusion_align_weight=0.5)
    a = torch.from_numpy(g["a_emb"]).cuda()
    v = torch.from_numpy(g["v_emb"]).cuda()
    loss, _ = step(v, a, torch.from_numpy(g["labels"]).cuda())
    cls_l, con_l = step.last_losses
    assert abs(float(loss) - float(g["loss"])) < 1e-5
    assert abs(float(con_l) - float(g["align"])) < 1e-5
    assert abs(float(cls_l) + 0.5 * float(con_l) - float(loss)) < 1e-6
    assert m.semantic_alignment.logit_scale.grad is not None


def test_int8_with_emotion_prior_golden():
    """INT8 images of prior_net and the token-bias Linears (K = 136 zero-padded to 144) vs quantize_dynamic."""
    from multimodalemotionrecognition_amd.int8 import quantize_dynamic_hip

    g = golden("int8_head_prior_b64.npz")
    m = head_model("concat", True).eval()
    q = quantize_dynamic_hip(m)
    assert sorted(q) == sorted(int8_ref.XATTN_INT8["concat"] + int8_ref.PRIOR_INT8)
    v, a = feats(64, 8, 149, seed=22)
    with torch.inference_mode():
        lq = m.xattn_from_features(v, a).cpu().numpy()
    diff = np.abs(lq - g["logits_int8"]).max()
    print("int8+prior head max|dlogit| vs reference:", diff)
    assert diff < 1e-2
    assert (lq.argmax(1) == g["logits_int8"].argmax(1)).mean() >= 62 / 64
    p = int8_ref.quantize_params(xattn_params("concat", True), int8_ref.XATTN_INT8["concat"] + int8_ref.PRIOR_INT8)
    vv, aa = params.feature_inputs(64, 8, 149, seed=22)
    lo, _ = fusion_ref.xattn_forward(p, torch.from_numpy(vv), torch.from_numpy(aa), use_prior=True)
    assert np.abs(lq - lo.numpy()).max() < 1e-2


@pytest.mark.parametrize("dim", [512, 768])
def test_encoder_width_transformer_pooling_golden(dim):
    """VideoNet.encode / WavLMAudioEncoder.encode pooling at head_dim 128 / 192: forward and gradients."""
    from multimodalemotionrecognition_amd.temporal import TemporalPooler

    g = golden(f"temporal_transformer_d{dim}.npz")
    pool = TemporalPooler(dim, "transformer", 4, 1, 0.1)
    sd = pool.state_dict()
    pool.load_state_dict({k: torch.from_numpy(params.init_tensor(k, tuple(v.shape), 0)) for k, v in sd.items()})
    pool = pool.cuda().eval()
    x = torch.from_numpy(g["x"]).cuda().requires_grad_(True)
    y = pool(x)
    assert max_abs(y, g["y"]) < 1e-4
    from multimodalemotionrecognition_amd.nn_ops import hip_linear  # noqa: F401 (product ops only below)
    w = torch.from_numpy(g["w"]).cuda()
    # d(sum(y * w))/dy = w: backprop the constant through the pooler's own autograd node
    y.backward(w)
    gx = g["grad_x"]
    assert max_abs(x.grad, gx) < 1e-4 * max(1.0, float(np.abs(gx).max()))
    for n, q in pool.named_parameters():
        if n == "pool.pool.score.4.bias":  # mathematically zero (softmax shift invariance)
            continue
        check_grad(g, n, q.grad.cpu(), atol=1e-4)


def test_gated_modality_dropout_leaves_dropped_branch_untouched():
    """fusion.py:47-53, 430: a dropped modality's projection output is zeros_like -> no gradient for
    audio_proj / video_proj and the encoder behind it; torch Adam skips them (no decay, no step count)."""
    from multimodalemotionrecognition_amd.fusion import FusionModel
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, make_loss

    torch.manual_seed(0)
    m = FusionModel(_Enc(768), _Enc(512), num_classes=8, mode="gated").cuda().train()
    opt = build_optimizer(m)
    step = TrainStep(m, opt, make_loss("gated"), "gated")
    m.modality_dropout.draw = lambda: (True, False)  # force: drop audio, keep video
    a = torch.randn(4, 768, device="cuda", requires_grad=True)
    v = torch.randn(4, 512, device="cuda", requires_grad=True)
    before = {n: q.detach().clone() for n, q in m.named_parameters()}
    step(v, a, torch.randint(0, 8, (4,), device="cuda"))
    for n, q in m.named_parameters():
        moved = not torch.equal(before[n], q.detach())
        assert moved == (not n.startswith("audio_proj.")), n
    assert a.grad is None and v.grad is not None
    names = {id(q): n for n, q in m.named_parameters()}
    steps = dict(zip([names[id(q)] for q in opt.param_groups[0]["params"]], opt.state_steps()[0]))
    assert steps["audio_proj.weight"] == 0 and steps["video_proj.weight"] == 1
