"""Isolated timing of the xattn head (C2 shapes: B=32, T=8, Ta=149, WavLM-base features): forward + backward,
fused (csrc/xattn_fused*.hip) vs the unfused schedule, each as a captured graph replayed back-to-back on an
otherwise idle GPU.  In the train step the head overlaps the next batch's WavLM forward (prefetch stream), so
its kernels' trace durations there include waiting for CUs; this tool gives the uncontended cost.
    python tools/bench_head.py [--iters 200] [--head concat|gated]"""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--head", default="concat")
    ap.add_argument("--train", type=int, default=1)
    ap.add_argument("--f1-pair", type=int, default=1)
    ap.add_argument("--wgrad-rows", type=int, default=0)
    ap.add_argument("--fused-only", type=int, default=0)
    args = ap.parse_args()
    from multimodalemotionrecognition_amd import xattn_fused as XF
    from multimodalemotionrecognition_amd import xattn_head as XH
    from multimodalemotionrecognition_amd.fusion import _head_grads
    from tests.gpu_helpers import feats, head_model
    XF.F1_PAIR = bool(args.f1_pair)
    if args.wgrad_rows:
        XF.WGRAD_ROWS = args.wgrad_rows

    m = head_model(args.head, False).train(bool(args.train))
    names, params = m.head_params()
    p = dict(zip(names, params))
    cfg = m.head_config()
    v, a = feats(32, 8, 149, seed=7)
    a = a.to(torch.bfloat16)
    rng = torch.full((1,), 4242, dtype=torch.int64, device="cuda")
    grads = {n: torch.zeros_like(t) for n, t in _head_grads(p, set(XH.used_param_names(cfg))).items()}
    dl = torch.from_numpy(np.random.default_rng(1).standard_normal((32, 8)).astype(np.float32)).cuda()
    res = {}
    for fused in ((True,) if args.fused_only else (False, True)):
        XF.ENABLED = fused

        def step():
            logits, ctx = XH.head_forward(p, cfg, v, a, bool(args.train), rng)
            XH.head_backward(p, ctx, dl[:, :logits.shape[1]].contiguous(), grads, need_dv_feat=True)

        def fwd():
            XH.head_forward(p, cfg, v, a, bool(args.train), rng)

        out = {}
        for name, fn in (("fwd", fwd), ("fwd+bwd", step)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.graph(g, stream=s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            for _ in range(5):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.iters):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) / args.iters * 1e3
        res["fused" if fused else "unfused"] = out
        print(("fused  " if fused else "unfused"), " ".join(f"{k} {v:7.1f} us" for k, v in out.items()), flush=True)
    XF.ENABLED = True


if __name__ == "__main__":
    main()
