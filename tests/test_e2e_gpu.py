"""End-to-end parity of the north-star path: full FusionModel(xattn) with WavLM-base + ResNet18 trunk +
head, train step (C2 semantics at B=2) and batch inference (C5 semantics), vs the fp32 CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import fusion_ref, int8_ref, resnet18_ref, train_ref, wavlm_ref
from oracle import params as OP

pytestmark = pytest.mark.gpu

B = 2


def _oracle_state():
    shapes = [("video_model." + n, s) for n, s in resnet18_ref.param_shapes()]
    shapes += [("audio_model.wavlm." + n, s) for n, s in wavlm_ref.wavlm_param_shapes()]
    shapes += fusion_ref.xattn_head_param_shapes()
    return {k: torch.from_numpy(v) for k, v in OP.init_state(shapes).items()}


def _model(p, xattn_head="concat"):
    from multimodalemotionrecognition_amd.train import build_model

    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True, xattn_head=xattn_head)
    sd = m.state_dict()
    missing = [k for k in p if k not in sd]
    assert not missing, missing[:5]
    for k, v in p.items():
        assert tuple(sd[k].shape) == tuple(v.shape), k
    m.load_state_dict({k: v.clone() for k, v in p.items()}, strict=False)
    return m.cuda()


def _clips(seed=11):
    v, a, y = OP.clip_inputs(B, seed=seed)
    return torch.from_numpy(v), torch.from_numpy(a), torch.from_numpy(y)


def test_train_step_vs_oracle():
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, make_loss

    p = _oracle_state()
    m = _model(p)
    # the oracle step has no dropout / drop-path: switch them off on the HIP model
    m.attn_dropout = 0.0
    m.v_drop_path.drop_prob = m.a_drop_path.drop_prob = 0.0
    m.xattn_mlp[2].p = 0.0
    m.audio_model.wavlm.train_semantics = False  # WavLM train-mode randomness: tests/test_wavlm_train_gpu.py
    opt = build_optimizer(m, lr=1e-3, weight_decay=1e-4)
    step = TrainStep(m, opt, make_loss("xattn"), "xattn")
    video, audio, labels = _clips()
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    loss, _ = step(video.cuda(), audio.cuda(), labels.cuda())
    torch.cuda.synchronize()

    trainable = [k for k in p if (k.startswith("video_model.") and not k.endswith(
        ("running_mean", "running_var", "num_batches_tracked"))) or
        (not k.startswith(("video_model.", "audio_model.")) and not k.startswith("audio_time_conv"))]
    for k in trainable:
        p[k].requires_grad_(True)
    ropt = train_ref.AdamRef([p[k] for k in trainable], lr=1e-3, weight_decay=1e-4)
    rloss = train_ref.train_step(p, trainable, ropt, video, audio, labels)
    print("loss hip/oracle", float(loss), rloss)
    assert abs(float(loss) - rloss) < 2e-2

    after = m.state_dict()
    # train-mode BN side effects (running stats, counter) match the oracle's
    for k in ("video_model.backbone.1.running_mean", "video_model.backbone.7.1.bn2.running_var"):
        d = float((after[k].cpu() - p[k]).abs().max())
        assert d < 2e-2 * max(1.0, float(p[k].abs().max())), (k, d)
    assert int(after["video_model.backbone.1.num_batches_tracked"]) == int(p["video_model.backbone.1.num_batches_tracked"]) == 1
    # first Adam step is ~ -lr*sign(g): compare update directions
    for k, lo in (("xattn_mlp.3.weight", 0.97), ("v_in_proj.weight", 0.9), ("video_model.backbone.7.1.conv2.weight", 0.75),
                  ("video_model.backbone.0.weight", 0.75)):
        dh = (after[k].cpu() - before[k].cpu()).flatten()
        dr = (p[k].detach() - torch.from_numpy(OP.init_state([(k, tuple(p[k].shape))])[k])).flatten()
        agree = float(((dh > 0) == (dr > 0)).float().mean())
        print(k, "update-sign agreement", agree)
        assert agree >= lo, (k, agree)
    # frozen encoder untouched
    k = "audio_model.wavlm.encoder.layers.0.attention.q_proj.weight"
    assert torch.equal(after[k], before[k])
    # second step: its forward must see the Adam-updated conv weights (the bf16 weight packs are derived
    # copies; a stale pack shows up as a loss that stays at the first step's value)
    loss2, _ = step(video.cuda(), audio.cuda(), labels.cuda())
    rloss2 = train_ref.train_step(p, trainable, ropt, video, audio, labels)
    print("step-2 loss hip/oracle", float(loss2), rloss2)
    assert abs(float(loss2) - rloss2) < 2e-2


@pytest.mark.parametrize("int8", [False, True])
def test_runner_predict_probs_vs_oracle(int8, tmp_path):
    """TorchModelRunner.predict_probs (optimized_runtime.py:99-108) through a reference-format checkpoint."""
    from multimodalemotionrecognition_amd.optimized_runtime import TorchModelRunner, process_batch

    p = _oracle_state()
    m = _model(p)
    ck = tmp_path / "best.pt"
    torch.save({"model": {k: v.cpu() for k, v in m.state_dict().items()}, "val_f1": 0.5,
                "config": {"fusion": "xattn", "xattn_head": "concat", "use_wavlm": True, "num_classes": 8}}, ck)
    del m
    r = TorchModelRunner(str(ck), device="cuda", enable_dynamic_quant=int8)
    video, audio, _ = _clips(seed=12)
    probs = r.predict_probs(video, audio)
    assert probs.device.type == "cpu" and tuple(probs.shape) == (B, 8)
    assert torch.allclose(probs.sum(1), torch.ones(B), atol=1e-5)
    q = int8_ref.quantize_params(p, int8_ref.XATTN_INT8["concat"]) if int8 else p
    with torch.no_grad():
        logits = train_ref.model_forward(q, video, audio, bn_training=False)
    ref = torch.softmax(logits, dim=1)
    d = float((probs - ref).abs().max())
    print("runner int8" if int8 else "runner bf16", "max|dprob|", d)
    assert d < (1e-2 if int8 else 5e-3)
    rows = process_batch(r, list(video), list(audio))
    assert [row["top1"]["label"] for row in rows] == [r.labels[i] for i in probs.argmax(1).tolist()]


@pytest.mark.parametrize("fusion", ["late", "concat", "gated"])
def test_non_xattn_train_steps_full_encoders(fusion):
    """C4 heads with the real encoders (ResNet18 trunk + frozen WavLM, B=2 3 s clips): full train steps run on
    the HIP path (late: NLL of the averaged softmaxes through both encoder classifiers, train.py:212-214) and
    the loss decreases on a repeated batch."""
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, build_model, make_loss

    torch.manual_seed(0)
    m = build_model(8, fusion, pretrained_video=False, use_wavlm=True).cuda()
    step = TrainStep(m, build_optimizer(m), make_loss(fusion), fusion)
    video, audio, labels = OP.clip_inputs(2, seed=4)
    video, audio, labels = torch.from_numpy(video).cuda(), torch.from_numpy(audio).cuda(), torch.from_numpy(labels).cuda()
    losses = [float(step(video, audio, labels)[0]) for _ in range(4)]
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("fusion", ["late", "gated"])
def test_non_xattn_prefetch_matches_inline(fusion):
    """FusionModel.prefetch_audio for late / concat / gated: the frozen WavLM hidden states of the next batch run
    ahead on the side stream; losses must equal the inline schedule bit for bit."""
    from multimodalemotionrecognition_amd.train import TrainStep, build_optimizer, build_model, make_loss

    video, audio, labels = OP.clip_inputs(2, seed=5)
    video, audio, labels = torch.from_numpy(video).cuda(), torch.from_numpy(audio).cuda(), torch.from_numpy(labels).cuda()
    runs = []
    for prefetch in (False, True):
        torch.manual_seed(0)
        m = build_model(8, fusion, pretrained_video=False, use_wavlm=True).cuda()
        step = TrainStep(m, build_optimizer(m), make_loss(fusion), fusion)
        torch.manual_seed(1)
        runs.append([float(step(video, audio, labels, next_audio=audio if prefetch else None)[0]) for _ in range(4)])
    assert runs[0] == runs[1], runs


@pytest.fixture(scope="module")
def c5_oracle():
    """The C5 workload (BASELINE.json configs[4]): one B=64 batch of 3 s clips through the fp32 oracle in eval
    mode, fp32 and with the head Linears quantized as quantize_dynamic({nn.Linear}) does (int8_ref)."""
    p = _oracle_state()
    video, audio, _ = OP.clip_inputs(64, seed=20261015)
    video, audio = torch.from_numpy(video), torch.from_numpy(audio)
    out = {}
    with torch.no_grad():
        vf, hidden = train_ref.encoders_forward(p, video, audio, bn_training=False)
        for int8 in (False, True):
            q = int8_ref.quantize_params(p, int8_ref.XATTN_INT8["concat"]) if int8 else p
            logits, _ = fusion_ref.xattn_forward(q, vf, hidden)
            out[int8] = torch.softmax(logits, dim=1)
    return p, video, audio, out


@pytest.mark.parametrize("int8", [False, True])
def test_runner_c5_b64_full_clips_vs_oracle(int8, c5_oracle, tmp_path):
    """C5 at its own workload: inference_worker.py:131-147 -> TorchModelRunner.predict_probs
    (optimized_runtime.py:95-108) on a [64,8,3,112,112] + [64,1,48000] batch, bf16 encoders and fp32 / INT8 head
    vs the oracle's forward.  Bars: probabilities 5e-3 (bf16) / 1e-2 (INT8) max-abs; top-1 agreement >= 0.95 of
    rows (random init gives near-uniform probabilities, so a row whose top-2 gap is below the probability error
    may flip; rows with a top-2 gap >= 2x the bar must all agree)."""
    from multimodalemotionrecognition_amd.optimized_runtime import TorchModelRunner, process_batch

    p, video, audio, ref = c5_oracle
    m = _model(p)
    ck = {"model": {k: v.cpu() for k, v in m.state_dict().items()}, "val_f1": 0.5,
          "config": {"fusion": "xattn", "xattn_head": "concat", "use_wavlm": True, "num_classes": 8}}
    del m
    r = TorchModelRunner(checkpoint=ck, device="cuda", enable_dynamic_quant=int8)
    probs = r.predict_probs(video, audio)
    ref = ref[int8]
    assert tuple(probs.shape) == (64, 8) and torch.allclose(probs.sum(1), torch.ones(64), atol=1e-5)
    d = float((probs - ref).abs().max())
    bar = 1e-2 if int8 else 5e-3
    agree = float((probs.argmax(1) == ref.argmax(1)).float().mean())
    top2 = ref.topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) >= 2 * bar
    print("C5", "int8" if int8 else "bf16", "max|dprob|", d, "top-1 agreement", agree, "clear rows", int(clear.sum()))
    assert d < bar
    assert agree >= 0.95
    assert bool((probs.argmax(1) == ref.argmax(1))[clear].all())
    rows = process_batch(r, list(video), list(audio))
    assert [row["top1"]["label"] for row in rows] == [r.labels[i] for i in probs.argmax(1).tolist()]
