"""Standalone timing of the batched weight-gradient fold (mer_wgrad_fold_batch) on the ResNet18 trunk's slabs at B = 32.

Launches the split-K partial pass of every trunk conv's weight gradient once (K.conv_wgrad(..., defer=folds), the
train step's shapes and split counts), then times the ONE fold launch of all records (the block segment's flush) with
HIP events, replaying the same record table N times.  Compare libraries with MER_HIP_LIB=<alt build>.
    python tools/bench_fold.py [--iters 20]
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd import kernels as K  # noqa: E402


def trunk_wgrad_shapes(N=256):
    """(x shape, dy shape, R, stride, pad) of every block conv's weight gradient (the stem's record is separate)."""
    out = []
    h, c = 28, 64
    for cout, s in ((64, 1), (128, 2), (256, 2), (512, 2)):
        ho = (h + 2 - 3) // s + 1
        out.append(((N, h, h, c), (N, ho, ho, cout), 3, s, 1))  # block 0 conv1
        out.append(((N, ho, ho, cout), (N, ho, ho, cout), 3, 1, 1))  # block 0 conv2
        if s == 2:
            out.append(((N, h, h, c), (N, ho, ho, cout), 1, s, 0))  # downsample
        out.append(((N, ho, ho, cout), (N, ho, ho, cout), 3, 1, 1))  # block 1 conv1
        out.append(((N, ho, ho, cout), (N, ho, ho, cout), 3, 1, 1))  # block 1 conv2
        h, c = ho, cout
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    folds = K.WgradFolds()
    keep = []
    for xs, ds, R, s, p in trunk_wgrad_shapes():
        x = torch.randn(*xs, device=dev).bfloat16()
        dy = torch.randn(*ds, device=dev).bfloat16()
        dw = torch.zeros(ds[-1], xs[-1], R, R, device=dev)
        K.conv_wgrad(x, dy, dw, R, R, s, p, defer=folds)
        keep += [x, dy, dw]
    rows, kept = list(folds.rows), list(folds.keep)
    slab_bytes = sum(int(t.numel()) * 4 for t in kept[0::3])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for it in range(a.iters + 3):
        folds.rows, folds.keep = list(rows), list(kept)
        if it == 3:
            torch.cuda.synchronize()
            ev[0].record()
        folds.flush()
    ev[1].record()
    torch.cuda.synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / a.iters
    print(f"records {len(rows)}  slab bytes {slab_bytes / 1e6:.1f} MB  fold {us:.1f} us  "
          f"{slab_bytes / us / 1e6:.2f} TB/s")


if __name__ == "__main__":
    main()
