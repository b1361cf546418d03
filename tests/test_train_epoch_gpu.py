"""The training entry point over the build's own loader: ``train_one_epoch`` (train.py:185-244)
driven by ``data.ClipLoader`` (decoded frames + WAV files -> device batches, the reference's (video, audio, label,
meta) 4-tuples of ravdess.py:616/654), with its one-batch lookahead prefetch of the next batch's frozen WavLM
forward and a cosine ``LambdaLR`` (train.py:1036-1047 shape) stepped per epoch over ``FusedAdam``.

Bar: bit-identical losses, predictions and final weights vs an explicit ``TrainStep`` loop over the same batches
in the same order with the same RNG stream (dropouts on, train mode)."""
import math

import numpy as np
import pytest
import torch

from oracle import io_ref as R

pytestmark = pytest.mark.gpu

B, NB, EPOCHS = 4, 3, 2


def _items(tmp_path):
    rng = np.random.default_rng(31)
    items = []
    for i in range(B * NB):
        T, H, W = int(rng.integers(10, 30)), int(rng.integers(96, 160)), int(rng.integers(96, 160))
        fp = tmp_path / f"f{i}.npy"
        np.save(fp, rng.integers(0, 256, (T, H, W, 3), dtype=np.uint8))
        wp = tmp_path / f"a{i}.wav"
        R.write_wav(wp, rng.uniform(-0.5, 0.5, (int(16000 * rng.uniform(2.0, 3.5)), 1)), 16000, "pcm16")
        items.append((str(fp), str(wp), int(rng.integers(0, 8)), None, {"actor": f"{i % 4:02d}"}))
    return items


def _model():
    from multimodalemotionrecognition_amd.train import build_model, build_optimizer

    torch.manual_seed(0)
    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda()
    opt = build_optimizer(m, lr=1e-3, weight_decay=1e-4)
    lam = lambda e: 0.5 * (1 + math.cos(math.pi * e / EPOCHS))  # noqa: E731  cosine over the epochs
    return m, opt, torch.optim.lr_scheduler.LambdaLR(opt, lam)


def _loader(items):
    from multimodalemotionrecognition_amd.data import ClipLoader

    return ClipLoader(items, batch_size=B, workers=4, shuffle=True, seed=3, augment=True)


def _recording_loss():
    from multimodalemotionrecognition_amd.losses import CrossEntropyLoss

    class Rec(CrossEntropyLoss):
        def __init__(self):
            super().__init__()
            self.seen = []

        def forward(self, logits, labels):
            loss = super().forward(logits, labels)
            self.seen.append(loss.detach().clone())
            return loss

    return Rec()


def test_train_one_epoch_over_clip_loader_matches_explicit_steps(tmp_path):
    from multimodalemotionrecognition_amd.train import TrainStep, train_one_epoch

    items = _items(tmp_path)
    dev = torch.device("cuda")

    # (a) the entry point
    m, opt, sched = _model()
    loader = _loader(items)
    assert len(loader) == NB
    torch.manual_seed(1)
    stats, lrs = [], []
    rec_a = _recording_loss()
    for _ in range(EPOCHS):
        lrs.append(opt.param_groups[0]["lr"])
        stats.append(train_one_epoch(m, loader, opt, dev, rec_a, "xattn"))
        sched.step()
    flat_a = [f.clone() for f in opt.flat_params()]
    assert lrs[1] < lrs[0]

    # (b) the same batches (a fresh loader replays the same epochs), explicit TrainStep with the same lookahead
    m2, opt2, sched2 = _model()
    loader2 = _loader(items)
    epochs = [[(v.clone(), a.clone(), y.clone()) for v, a, y, meta in loader2] for _ in range(EPOCHS)]
    for meta_epoch in range(EPOCHS):
        assert len(epochs[meta_epoch]) == NB
    assert not torch.equal(epochs[0][0][2], epochs[1][0][2]) or not torch.equal(epochs[0][0][1], epochs[1][0][1])
    rec_b = _recording_loss()
    step = TrainStep(m2, opt2, rec_b, "xattn")
    torch.manual_seed(1)
    for e, batches in enumerate(epochs):
        tot, preds, ys = 0.0, [], []
        losses = []
        for i, (v, a, y) in enumerate(batches):
            nxt = batches[i + 1][1] if i + 1 < len(batches) else None
            loss, pred = step(v, a, y, next_audio=nxt)
            losses.append(loss * y.numel())
            preds.append(pred)
            ys.append(y)
        tot = float(torch.stack(losses).sum().cpu()) / (B * NB)
        acc = float((torch.cat(preds) == torch.cat(ys)).float().mean())
        print("epoch", e, "entry point", stats[e]["loss"], stats[e]["acc"], "explicit", tot, acc)
        print("per-step losses", [float(x) for x in rec_a.seen], [float(x) for x in rec_b.seen])
        assert stats[e]["loss"] == tot, (e, stats[e]["loss"], tot)
        assert stats[e]["acc"] == acc
        sched2.step()
    for a, b in zip(flat_a, opt2.flat_params()):
        assert torch.equal(a, b), float((a - b).abs().max())
    assert all(np.isfinite(s["loss"]) for s in stats)
