"""Where do the non-HIP-kernel launches of a train step come from (copies, fills)?  Runs 3 steps of
bench.py's workload under torch.profiler and prints the aten ops that own copy/fill launches, with the
innermost python frames of this package."""
import sys
from collections import Counter
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from multimodalemotionrecognition_amd.train import TrainStep, build_model, build_optimizer, make_loss  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).to(dev)
    opt = build_optimizer(model, lr=1e-3, weight_decay=1e-4)
    step = TrainStep(model, opt, make_loss("xattn"), "xattn")
    video, audio, labels = bench.synthetic_batch(dev, 1)
    for _ in range(3):
        step(video, audio, labels)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True) as prof:
        for _ in range(3):
            step(video, audio, labels)
        torch.cuda.synchronize()
    c = Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::clone", "aten::contiguous",
                       "aten::to", "aten::_to_copy", "aten::cat", "aten::stack", "aten::add_", "aten::mul"):
            frames = [f for f in (ev.stack or []) if "multimodalemotionrecognition_amd" in f or "bench" in f]
            c[(ev.name, " <- ".join(frames[:3]))] += 1
    for (name, where), n in c.most_common(40):
        print(f"{n / 3:6.1f}/step  {name:18s} {where}")


if __name__ == "__main__":
    main()
