"""Standalone frozen WavLM-base forward at the C2 shape (B=32, 48,000 samples): the captured graph replayed
back-to-back on an otherwise idle GPU (train-mode semantics as in the train step, or eval).  Run it under
rocprofv3 --kernel-trace --stats for the per-kernel durations without the trunk stream's contention.
    python tools/bench_wavlm.py [--iters 20] [--eval]"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--eval", action="store_true")
    args = ap.parse_args()
    from multimodalemotionrecognition_amd.wavlm_audio import WavLMAudioEncoder
    from oracle import params as OP

    torch.manual_seed(0)
    enc = WavLMAudioEncoder(num_classes=8).cuda()
    enc.train(not args.eval)
    _, a, _ = OP.clip_inputs(args.batch, seed=3)
    a = torch.from_numpy(a).cuda()
    for _ in range(3):
        enc.encode_sequence(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        enc.encode_sequence(a)
    e1.record()
    torch.cuda.synchronize()
    print(f"WavLM forward B={args.batch} {'eval' if args.eval else 'train-mode'}: "
          f"{e0.elapsed_time(e1) / args.iters:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
