"""Is the bench train step host-bound?  Times, for the bench's TrainStep (B=32, xattn, WavLM prefetch):
  - idle-start: from an idle GPU, the host time to enqueue one step vs the time until the GPU has finished it;
  - steady state: 50 back-to-back steps, the host's average enqueue time per step vs the wall time per step.
If the steady-state host time per step is ~ the wall time per step, the GPU waits for the host and kernel-side
savings do not show in steps/s.  python tools/host_step.py"""
import sys
import time
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
    step = TrainStep(model, opt, make_loss("xattn"), "xattn", None)
    video, audio, labels = bench.synthetic_batch(dev, 20261015)
    for _ in range(10):
        step(video, audio, labels, next_audio=audio)
    torch.cuda.synchronize()
    for i in range(5):
        t0 = time.perf_counter()
        step(video, audio, labels, next_audio=audio)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"idle-start step {i}: host enqueue {1e3 * (t1 - t0):.3f} ms, done after {1e3 * (t2 - t0):.3f} ms")
    n = 50
    host = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        a = time.perf_counter()
        step(video, audio, labels, next_audio=audio)
        host.append(time.perf_counter() - a)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"steady: host {1e3 * sum(host) / n:.3f} ms/step (min {1e3 * min(host):.3f}, max {1e3 * max(host):.3f}), "
          f"enqueue of {n} done at {1e3 * (t1 - t0):.1f} ms, GPU done at {1e3 * (t2 - t0):.1f} ms "
          f"-> {1e3 * (t2 - t0) / n:.3f} ms/step")


if __name__ == "__main__":
    main()
