"""How much of the bench train step is the main stream on its own?  Times the bench's TrainStep (B=32, xattn,
next-batch WavLM prefetch) as is, then with the prefetched WavLM forward replaced by a cached copy of its output
(the side stream then runs no encoder work: the main stream's trunk / head / backward / Adam alone), then as is
again.  The gap between the two is what the concurrent WavLM stream costs the critical path.
    python tools/no_wavlm_step.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from multimodalemotionrecognition_amd.train import TrainStep, build_model, build_optimizer, make_loss  # noqa: E402


def timed(step, batch, n=50):
    video, audio, labels = batch
    for _ in range(5):
        step(video, audio, labels, next_audio=audio)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        step(video, audio, labels, next_audio=audio)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).to(dev)
    opt = build_optimizer(model, lr=1e-3, weight_decay=1e-4)
    step = TrainStep(model, opt, make_loss("xattn"), "xattn", None)
    batch = bench.synthetic_batch(dev, 20261015)
    for _ in range(10):
        step(*batch, next_audio=batch[1])
    print(f"with the WavLM stream:    {timed(step, batch):.3f} ms/step")
    enc = model.audio_model.encode_sequence
    cache = {}

    def cached(audio, *a, **k):  # the encoder's output, computed once, then served without any kernel
        if "out" not in cache:
            cache["out"] = enc(audio, *a, **k)
            cache["out"] = tuple(t.clone() for t in cache["out"]) if isinstance(cache["out"], tuple) \
                else cache["out"].clone()
        return cache["out"]

    model.audio_model.encode_sequence = cached
    print(f"main stream alone:        {timed(step, batch):.3f} ms/step")
    model.audio_model.encode_sequence = enc
    print(f"with the WavLM stream:    {timed(step, batch):.3f} ms/step")


if __name__ == "__main__":
    main()
