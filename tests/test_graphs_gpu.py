"""Captured hipGraphs (graphs.py) replay exactly the eager launch schedule.

* WavLM forward: graph replays agree with the eager forward as closely as two eager runs agree.
* Full train step (ResNet18 trunk fwd/bwd graphs + eager head + FusedAdam): loss and gradients match the
  eager schedule at identical weights within fp32 reassociation noise (the BatchNorm statistics use
  striped fp32 atomics, so bitwise equality is not expected); BN running statistics advance once per step.
* Audio prefetch: the next batch's WavLM features (computed during the backward) are bit-identical.
"""
import pytest
import torch

import bench
from multimodalemotionrecognition_amd import graphs as G

pytestmark = pytest.mark.gpu


def _rel_rms(a, b):
    a, b = a.float(), b.float()
    return float((a - b).pow(2).mean().sqrt() / b.pow(2).mean().sqrt().clamp_min(1e-12))


def test_wavlm_graph_replay_matches_eager():
    """The GroupNorm statistics of conv0 are fp32 atomics, so two eager runs already differ by bf16
    rounding flips: graph replays must agree with eager runs as closely as eager runs agree with
    each other (and far inside the 2e-2 parity bar of the WavLM path)."""
    from multimodalemotionrecognition_amd.wavlm_audio import WavLMBackbone

    torch.manual_seed(0)
    m = WavLMBackbone().cuda().eval()
    wav = (0.1 * torch.randn(4, 48000, device="cuda")).clamp(-1, 1)
    prev = G.ENABLED
    try:
        G.ENABLED = False
        e1, e2 = m.forward_hip(wav), m.forward_hip(wav)
        noise = _rel_rms(e1, e2)
        G.ENABLED = True
        outs = [m.forward_hip(wav) for _ in range(4)]  # eager, capture+replay, replay, replay
        assert len(m._graphs.graphs) == 1
        for o in outs[1:]:
            assert _rel_rms(o, e1) <= max(4 * noise, 2e-3)
        wav2 = (0.1 * torch.randn(4, 48000, device="cuda")).clamp(-1, 1)
        G.ENABLED = False
        ref = m.forward_hip(wav2)
        G.ENABLED = True
        assert _rel_rms(m.forward_hip(wav2), ref) <= max(4 * noise, 2e-3)  # new input via the static buffer
    finally:
        G.ENABLED = prev


def _twin(seed):
    from multimodalemotionrecognition_amd.train import TrainStep, build_model, build_optimizer, make_loss

    torch.manual_seed(seed)
    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    # no stochastic ops: dropout / drop-path off so the two schedules see identical math
    m.attn_dropout = 0.0
    m.v_drop_path.drop_prob = m.a_drop_path.drop_prob = 0.0
    m.xattn_mlp[2].p = 0.0
    m.audio_model.wavlm.train_semantics = False  # (train-mode WavLM graphs: tests/test_wavlm_train_gpu.py)
    opt = build_optimizer(m)
    return m, TrainStep(m, opt, make_loss("xattn"), "xattn")


def test_train_step_graphs_match_eager():
    """Graphed train step vs the eager schedule at IDENTICAL weights: the graphed model runs three steps
    (eager, capture + replay, replay -- its Adam updates exercise the per-step weight re-packing inside
    the graphs), its state is copied into an eager twin, then both run one forward + backward on the same
    batch.  Every reduction of the step is fixed-order (no fp32 atomics), so the eager re-runs are
    bit-identical and the graphed step must reproduce them bit-for-bit."""
    prev = G.ENABLED
    try:
        G.ENABLED = True
        mg, sg = _twin(7)
        video, audio, labels = bench.synthetic_batch(torch.device("cuda"), 5)
        video, audio, labels = video[:4], audio[:4], labels[:4]
        for _ in range(3):
            sg(video, audio, labels)
        assert mg.video_model.backbone._graphs.graphs, "trunk graphs were not captured"
        assert mg.audio_model.wavlm._graphs.graphs, "WavLM graphs were not captured"
        assert int(mg.state_dict()["video_model.backbone.1.num_batches_tracked"]) == 3
        G.ENABLED = False
        me, se = _twin(8)
        me.load_state_dict(mg.state_dict())
        grads = {}
        for tag, m, st, on in (("graph", mg, sg, True), ("eager", me, se, False), ("eager2", me, se, False),
                               ("eager3", me, se, False)):
            G.ENABLED = on
            m.train()
            st.opt.zero_grad()
            loss = st.loss_fn(m(video, audio), labels)
            loss.backward()
            grads[tag] = (float(loss), {n: q.grad.detach().clone() for n, q in m.named_parameters()
                                        if q.grad is not None})
        (lg, gg), (le, ge), (le2, ge2), (_, ge3) = grads["graph"], grads["eager"], grads["eager2"], grads["eager3"]
        assert set(gg) == set(ge) and len(gg) > 60
        assert le == le2 and all(torch.equal(ge[n], ge2[n]) and torch.equal(ge[n], ge3[n]) for n in ge), \
            "eager train step is not run-to-run reproducible"
        worst = []
        for n in ge:
            den = max(float(ge[n].norm()), 1e-6)
            worst.append((float((gg[n] - ge[n]).norm()) / den, n))
        assert lg == le and all(d == 0.0 for d, _ in worst), (lg, le, sorted(worst)[-3:])
    finally:
        G.ENABLED = prev


@pytest.mark.parametrize("early", [False, True])
def test_audio_prefetch_matches_inline(early, monkeypatch):
    """TrainStep(next_audio=...) runs the frozen WavLM of the next batch on a side stream: from the top of this
    step's forward (early prefetch, FusionModel.queue_next_audio: this step keeps a copy of its own borrowed
    encoder output first) or during this step's backward.  The WavLM path is deterministic, so the prefetched
    features must be bit-identical to an inline encode of the same waveform; a prefetch is used only for the
    very tensor it was computed from."""
    from multimodalemotionrecognition_amd import train as T

    monkeypatch.setattr(T, "EARLY_PREFETCH", early)
    prev = G.ENABLED
    try:
        G.ENABLED = True
        mb, sb = _twin(11)
        video, audio, labels = bench.synthetic_batch(torch.device("cuda"), 6)
        v1, a1, y1 = video[:4], audio[:4].clone(), labels[:4]
        v2, a2, y2 = video[4:8], audio[4:8].clone(), labels[4:8]
        seen = []
        orig = mb.xattn_from_features
        mb.xattn_from_features = lambda v, a: (seen.append(a.detach().clone()), orig(v, a))[1]
        seq = [(v1, a1, y1), (v2, a2, y2), (v1, a1, y1)]
        for i, (v, a, y) in enumerate(seq):
            nxt = seq[i + 1][1] if i + 1 < len(seq) else None
            sb(v, a, y, next_audio=nxt)
        assert mb._prefetched is None  # consumed
        for (v, a, y), feats in zip(seq, seen):
            with torch.no_grad():
                ref = mb.audio_model.encode_sequence(a)
            assert torch.equal(feats, ref)
        # a prefetch for a tensor that is then modified in place is not used
        mb.prefetch_audio(a2)
        a2.mul_(0.5)
        seen.clear()
        sb(v2, a2, y2)
        with torch.no_grad():
            assert torch.equal(seen[0], mb.audio_model.encode_sequence(a2))
    finally:
        G.ENABLED = prev


@pytest.mark.parametrize("train", [False, True])
def test_head_graph_matches_eager(train):
    """xattn head alone (stub encoders, C2 feature shapes): graphed forward + backward reproduce the eager
    head bit-for-bit (every reduction is fixed-order: no fp32 atomics), with dropout masks drawn from the
    same host seeds in both modes."""
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss
    from multimodalemotionrecognition_amd.optim import FusedAdam
    from tests.gpu_helpers import feats, head_model

    prev = G.ENABLED
    try:
        v, a = feats(32, 8, 149, seed=7)
        labels = torch.arange(32, device="cuda") % 8
        runs = {}
        for on in (False, True):
            G.ENABLED = on
            m = head_model("concat", False).train(train)
            opt = FusedAdam([q for n, q in m.named_parameters() if not n.startswith(("audio_model", "video_model"))])
            for it in range(3):  # eager, capture + replay, replay
                opt.zero_grad()
                vv = v.clone().requires_grad_(True)
                torch.manual_seed(100 + it)
                loss = CrossEntropyLoss()(m.xattn_from_features(vv, a), labels)
                loss.backward()
            runs[on] = (float(loss), vv.grad.clone(),
                        {n: q.grad.clone() for n, q in m.named_parameters() if q.grad is not None})
            if on:
                assert m._head_graphs.graphs, "head graphs were not captured"
        (le, dve, ge), (lg, dvg, gg) = runs[False], runs[True]
        assert le == lg
        assert torch.equal(dve, dvg)
        assert set(ge) == set(gg)
        for n in ge:
            assert torch.equal(ge[n], gg[n]), n
    finally:
        G.ENABLED = prev
