"""C4 heads with the REAL encoders vs the fp32 oracle: late (fusion.py:358-363 through
WavLMAudioEncoder.forward wavlm_audio.py:121-144 and VideoNet.forward video.py:42-44), concat / gated
(fusion.py:413-435 through WavLMAudioEncoder.encode wavlm_audio.py:146-163 and VideoNet.encode video.py:34-40),
B=2 3 s clips, train-mode BatchNorm, deterministic variant (dropouts / ModalityDropout / WavLM train-mode
randomness off).

* the encoders' embeddings (``encode``: frame-mean of the bf16 ResNet18 features; WavLM frame-mean of the
  fp32-output ``encode_sequence(out_dtype=float32)``) and that fp32 hidden-state path itself;
* teacher-forced head: the HIP head on the HIP embeddings vs the oracle head on the SAME embeddings -- fp32 head
  parity (outputs, loss, every head gradient);
* the whole model's outputs and loss, and one full train step's loss / BN running statistics.
Bars are set from measurement (bf16 encoders vs the fp32 oracle); each assert states its bar."""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, train_ref
from oracle import params as OP

pytestmark = pytest.mark.gpu

B = 2


def _rel_rms(a, b):
    a, b = a.detach().float().cpu(), torch.as_tensor(b).detach().float().cpu()
    return float((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt().clamp_min(1e-30))


def _model_and_oracle(mode):
    from multimodalemotionrecognition_amd.train import build_model

    m = build_model(8, mode, pretrained_video=False, use_wavlm=True)
    sd = m.state_dict()
    p = {k: torch.from_numpy(OP.init_tensor(k, tuple(v.shape), 0)) for k, v in sd.items()}
    m.load_state_dict({k: v.clone() for k, v in p.items()})
    m = m.cuda().train()
    m.audio_model.wavlm.train_semantics = False
    m.audio_model.classifier[2].p = 0.0
    if mode == "concat":
        m.fusion[2].p = 0.0
    if mode == "gated":
        m.gate[2].p = 0.0
        m.modality_dropout.audio_dropout_p = m.modality_dropout.video_dropout_p = 0.0
    return m, p


def _clips(seed):
    v, a, y = OP.clip_inputs(B, seed=seed)
    return torch.from_numpy(v), torch.from_numpy(a), torch.from_numpy(y)


def test_encode_paths_vs_oracle():
    """encode_sequence(out_dtype=float32), WavLMAudioEncoder.encode, VideoNet.encode vs the oracle."""
    m, p = _model_and_oracle("concat")
    video, audio, _ = _clips(21)
    with torch.no_grad():
        hid32 = m.audio_model.encode_sequence(audio.cuda(), out_dtype=torch.float32)
        hid16 = m.audio_model.encode_sequence(audio.cuda())
        a_emb = m.audio_model.encode(audio.cuda())
        v_emb = m.video_model.encode(video.cuda())
    vf, hidden = train_ref.encoders_forward(p, video, audio, bn_training=True)
    ra = train_ref.audio_encode(p, hidden)
    rv = train_ref.video_encode(vf).detach()
    e_hid, e_a, e_v = _rel_rms(hid32, hidden), _rel_rms(a_emb, ra), _rel_rms(v_emb, rv)
    print(f"rel-RMS: hidden fp32 {e_hid:.3e}  a_emb {e_a:.3e}  v_emb {e_v:.3e}")
    assert hid32.dtype == torch.float32 and tuple(hid32.shape) == (B, 149, 768)
    assert e_hid < 5e-2  # bf16 WavLM, 12 layers (DESIGN §2 bar)
    assert e_a < 5e-2 and e_v < 3e-2
    # the bf16 output is the fp32 output rounded once (same arithmetic, different final store)
    assert _rel_rms(hid16.float(), hid32) < 4e-3


@pytest.mark.parametrize("mode", ["late", "concat", "gated"])
def test_teacher_forced_head_vs_oracle(mode):
    """HIP head on the HIP encoders' embeddings vs the oracle head on the same embeddings: fp32-class parity."""
    from multimodalemotionrecognition_amd import embedding_head as EH
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss, LateNLLLoss

    m, p = _model_and_oracle(mode)
    video, audio, labels = _clips(22)
    with torch.no_grad():
        hidden = m.audio_model.encode_sequence(audio.cuda(), out_dtype=torch.float32)
        vfeat = m.video_model.backbone(video.cuda().view(B * 8, 3, 112, 112)).view(B, 8, 512)
    hid = hidden.detach().clone()
    vf = vfeat.detach().clone()
    if mode == "late":
        a_in = hid.mean(1).requires_grad_(True)
        v_in = vf.mean(1).requires_grad_(True)
        from multimodalemotionrecognition_amd.nn_ops import hip_linear, hip_dropout  # noqa: F401
        h = hip_linear(a_in, m.audio_model.classifier[0], act="relu")
        a_logits = hip_linear(h, m.audio_model.classifier[3])
        v_logits = hip_linear(v_in, m.video_model.classifier)
        out = EH.late_probs(a_logits, v_logits)
        loss = LateNLLLoss()(out, labels.cuda())
    else:
        a_in = m.audio_model.temporal_pool(hid).detach().requires_grad_(True)
        v_in = m.video_model.temporal_pool(vf).detach().requires_grad_(True)
        out = EH.embedding_head(m, a_in, v_in)
        loss = CrossEntropyLoss()(out, labels.cuda())
    loss.backward()

    q = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in p.items()}
    ra = a_in.detach().cpu().clone().requires_grad_(True)
    rv = v_in.detach().cpu().clone().requires_grad_(True)
    if mode == "late":
        h = torch.relu(fusion_ref.linear(ra, q, "audio_model.classifier.0"))
        rout = fusion_ref.late_forward(fusion_ref.linear(h, q, "audio_model.classifier.3"),
                                       fusion_ref.linear(rv, q, "video_model.classifier"))
        rloss = fusion_ref.late_nll(rout, labels)
        names = ["audio_model.classifier.0.weight", "audio_model.classifier.3.weight", "video_model.classifier.weight",
                 "video_model.classifier.bias"]
    else:
        rout = fusion_ref.embedding_fusion_forward(q, mode, ra, rv)
        rloss = fusion_ref.cross_entropy(rout, labels)
        names = [n for n in p if n.startswith(("audio_proj", "video_proj", "fusion.", "gate.", "classifier."))]
    rloss.backward()
    d_out = float((out.detach().cpu() - rout.detach()).abs().max())
    print(mode, "teacher-forced max|d out|", d_out, "loss", float(loss.detach()), float(rloss.detach()))
    assert d_out < 1e-4 and abs(float(loss) - float(rloss)) < 1e-4
    pm = dict(m.named_parameters())
    for n in names:
        e = _rel_rms(pm[n].grad, q[n].grad)
        assert e < 1e-4, (n, e)
    assert _rel_rms(a_in.grad, ra.grad) < 1e-4 and _rel_rms(v_in.grad, rv.grad) < 1e-4


@pytest.mark.parametrize("mode", ["late", "concat", "gated"])
def test_full_model_and_train_step_vs_oracle(mode):
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, make_loss

    m, p = _model_and_oracle(mode)
    video, audio, labels = _clips(23)
    with torch.no_grad():
        out = m(video.cuda(), audio.cuda())
    ref = train_ref.embedding_model_forward(p, mode, video, audio, bn_training=True).detach()
    d = float((out.cpu() - ref).abs().max())
    print(mode, "full-model max|d out|", d, "scale", float(ref.abs().max()))
    # bf16 encoders vs fp32 oracle (the head is fp32): late = probabilities (measured 1.75e-3), concat / gated =
    # logits (measured 9.8e-3 / 9.5e-3)
    assert d < (5e-3 if mode == "late" else 3e-2), d

    m, p = _model_and_oracle(mode)  # fresh running statistics for the step
    opt = build_optimizer(m, lr=1e-3, weight_decay=1e-4)
    step = TrainStep(m, opt, make_loss(mode), mode)
    loss, pred = step(video.cuda(), audio.cuda(), labels.cuda())
    torch.cuda.synchronize()
    trainable = [n for n, q in m.named_parameters() if q.requires_grad and id(q) not in
                 {id(u) for u in m.unused_parameters()}]
    for n in trainable:
        p[n].requires_grad_(True)
    ropt = train_ref.AdamRef([p[n] for n in trainable], lr=1e-3, weight_decay=1e-4)
    rloss = train_ref.train_step_mode(p, trainable, ropt, mode, video, audio, labels)
    print(mode, "train-step loss hip/oracle", float(loss), rloss)
    assert abs(float(loss) - rloss) < 1e-2  # measured 1.7e-3 / 2.3e-3 / 3.6e-3 (late / concat / gated)
    assert pred.shape == (B,) and pred.dtype == torch.int64
    sd = m.state_dict()
    for k in ("video_model.backbone.1.running_mean", "video_model.backbone.7.1.bn2.running_var"):
        e = float((sd[k].cpu() - p[k]).abs().max()) / max(1.0, float(p[k].abs().max()))
        assert e < 5e-3, (k, e)
