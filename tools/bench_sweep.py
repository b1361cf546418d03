"""C4 (BASELINE.json configs[3]): the fusion-head sweep under one HIP backend -- full train steps (ResNet18 +
WavLM-base frozen + head, B=32 synthetic 3 s clips, fwd+bwd+Adam) for late / concat / gated / xattn /
xattn + emotion-prior bias, steps/s each.
    python tools/bench_sweep.py [--steps 30] [--warmup 10]"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import params  # noqa: E402  (synthetic clip generator only)
from multimodalemotionrecognition_amd.train import TrainStep, build_model, build_optimizer, make_loss  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=30)
ap.add_argument("--warmup", type=int, default=10)  # graphs are captured during the first steps
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--modes", default="late,concat,gated,xattn,xattn+prior")
args = ap.parse_args()
MODES = args.modes.split(",")
video, audio, labels = params.clip_inputs(args.batch, seed=20261015)
video, audio, labels = torch.from_numpy(video).cuda(), torch.from_numpy(audio).cuda(), torch.from_numpy(labels).cuda()
res = {}
for name, fusion, kw in (("late", "late", {}), ("concat", "concat", {}), ("gated", "gated", {}),
                         ("xattn", "xattn", {}), ("xattn+prior", "xattn", {"xattn_use_emotion_prior": True, "forward_emotion_prior_flags": True})):
    if name not in MODES:
        continue
    torch.manual_seed(0)
    model = build_model(8, fusion, pretrained_video=False, use_wavlm=True, **kw).cuda()
    if kw:  # the reference never forwards the prior flags (train.py:454-469); set the module up explicitly
        assert model.emotion_prior_bias is not None, "emotion prior requested but not built"
    step = TrainStep(model, build_optimizer(model), make_loss(fusion), fusion)
    nxt = audio  # every fusion mode prefetches the frozen WavLM output of the next batch
    for _ in range(args.warmup):
        step(video, audio, labels, next_audio=nxt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss, _ = step(video, audio, labels, next_audio=nxt)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    res[name] = {"ms_per_step": round(dt * 1e3, 3), "steps_per_s": round(1 / dt, 2), "loss": round(float(loss), 4)}
    del step, model
    torch.cuda.empty_cache()
print(json.dumps({"config": f"C4 fusion-head sweep, B={args.batch}, WavLM frozen", **res}))
