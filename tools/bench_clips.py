"""Time the device clip assembly (csrc/clips.hip) with HIP events: B=32 clips x 8 decoded RGB frames at a given
source size -> [32, 8, 3, 112, 112], and a ragged 32-waveform batch -> [32, 1, 48000].
    python tools/bench_clips.py [H W]"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd.clips import pad_crop_waveforms, video_clip_batch  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (720, 1280)
g = torch.Generator(device="cuda").manual_seed(0)
frames = torch.randint(0, 256, (32, 8, H, W, 3), dtype=torch.uint8, device="cuda", generator=g)
ms = timed(lambda: video_clip_batch(frames))
out_bytes = 32 * 8 * 3 * 112 * 112 * 4
src_bytes = 32 * 8 * 112 * 112 * 4 * 3  # 4 taps x 3 channels gathered per output pixel (upper bound, cached)
wavs = [torch.randn(40000 + 997 * i) for i in range(32)]
ms_w = timed(lambda: pad_crop_waveforms(wavs, device="cuda"), iters=20)
print(json.dumps({"frames_src": [H, W], "clip_batch_ms": round(ms, 4), "clips_per_s": round(32 / ms * 1e3, 1),
                  "frame_out_GBps": round(out_bytes / ms / 1e6, 1), "gathered_src_bytes": src_bytes,
                  "wav_batch_ms_incl_h2d": round(ms_w, 4)}))
