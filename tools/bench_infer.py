"""C5 (BASELINE.json configs[4]): inference_worker batch path at B=64 -- TorchModelRunner.predict_probs on
synthetic 3 s clips (resident on the GPU), bf16 encoders + fp32 head vs the INT8 dynamic-quantised Linear head
(quantize_dynamic mirror), clips/s for each and top-1 agreement between them.  Random-init weights (same
state dict for both runners).
    python tools/bench_infer.py [--batch 64] [--iters 20]"""
import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from oracle import params  # noqa: E402  (synthetic clip generator only)
from multimodalemotionrecognition_amd.optimized_runtime import TorchModelRunner  # noqa: E402
from multimodalemotionrecognition_amd.train import build_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--iters", type=int, default=20)
args = ap.parse_args()

torch.manual_seed(0)
model = build_model(8, "xattn", pretrained_video=False, use_wavlm=True)
ck = {"model": {k: v.detach().cpu() for k, v in model.state_dict().items()}, "val_f1": 0.0,
      "config": {"fusion": "xattn", "use_wavlm": True, "num_classes": 8}}
video, audio, _ = params.clip_inputs(args.batch, seed=20261015)
video, audio = torch.from_numpy(video).cuda(), torch.from_numpy(audio).cuda()
out = {"config": "C5 inference_worker batch, xattn + WavLM + ResNet18", "batch": args.batch}
probs = {}
for name, q in (("bf16", False), ("int8", True)):
    runner = TorchModelRunner(checkpoint=ck, device="cuda", enable_dynamic_quant=q)
    for _ in range(3):
        runner.predict_probs(video, audio)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        p = runner.predict_probs(video, audio)  # includes the probs D2H copy, like the reference's .cpu()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.iters
    probs[name] = p
    out[name] = {"ms_per_batch": round(dt * 1e3, 3), "clips_per_s": round(args.batch / dt, 1)}
out["top1_agreement_int8_vs_bf16"] = float((probs["int8"].argmax(1) == probs["bf16"].argmax(1)).float().mean())
out["max_abs_prob_diff"] = float((probs["int8"] - probs["bf16"]).abs().max())
print(json.dumps(out))
