"""Time every bf16 GEMM variant on the north-star's WavLM shapes (B=32): python tools/bench_gemm.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd import kernels as K  # noqa: E402

B = 32
SHAPES = {
    "conv1 (rows)": (B * 4799, 512, 1536, (4799, 1024, 9599 * 512), B * 9599 * 512),
    "conv2 (rows)": (B * 2399, 512, 1536, (2399, 1024, 4799 * 512), B * 4799 * 512),
    "conv3 (rows)": (B * 1199, 512, 1536, (1199, 1024, 2399 * 512), B * 2399 * 512),
    "conv4 (rows)": (B * 599, 512, 1536, (599, 1024, 1199 * 512), B * 1199 * 512),
    "conv5 (rows)": (B * 299, 512, 1024, (299, 1024, 599 * 512), B * 599 * 512),
    "conv6 (rows)": (B * 149, 512, 1024, (149, 1024, 299 * 512), B * 299 * 512),
    "qkv": (B * 149, 2304, 768, None, None),
    "ffn1": (B * 149, 3072, 768, None, None),
    "ffn2": (B * 149, 768, 3072, None, None),
    "out_proj": (B * 149, 768, 768, None, None),
    "f1pair": (B * 149, 256, 768, None, None),  # the fused head's F1 product against stacked hi/lo planes (fp32 out)
    "sq4096": (4096, 4096, 4096, None, None),
    "sq8192": (8192, 8192, 8192, None, None),
}
ONLY = next((a.split("=")[1].split(",") for a in sys.argv if a.startswith("--shapes=")), None)


VARIANTS = [int(v) for v in next((a.split("=")[1] for a in sys.argv if a.startswith("--variants=")),
                                  "0,7,9,13,18").split(",")]


def main():
    torch.manual_seed(0)
    quick = "--quick" in sys.argv  # profiling: fewer shapes / reps
    for name, (M, N, Kd, rows, alen) in SHAPES.items():
        if quick and name not in ("conv1 (rows)", "qkv", "ffn2"):
            continue
        if (ONLY is None and (name.startswith("sq") or name == "f1pair")) or (ONLY is not None and name.split()[0] not in ONLY):
            continue
        a = (torch.rand(alen if rows else M * Kd, device="cuda") * 2 - 1).bfloat16()
        if not rows:
            a = a.view(M, Kd)
        w = (torch.rand(N, Kd, device="cuda") * 2 - 1).bfloat16()
        outs = {}
        resid = "--resid32" in sys.argv  # the WavLM residual GEMMs: fp32 output + bf16 residual + bias
        r = (torch.rand(M, N, device="cuda") * 2 - 1).bfloat16() if resid else None
        bias = torch.rand(N, device="cuda") if resid else None
        gbias = bias if bias is not None else torch.rand(N, device="cuda")
        for odt in ((torch.float32,) if (resid or "--f32" in sys.argv) else (torch.bfloat16,)):
            for v in VARIANTS:
                out = torch.empty(M, N, device="cuda", dtype=odt)
                kw = dict(M=M, K=Kd, rows=rows) if rows else {}
                if resid:
                    kw.update(residual=r, bias=bias)
                if "--gelu" in sys.argv:  # bias + GELU epilogue (FFN-up, the feature-extractor convs)
                    kw.update(bias=gbias, act="gelu")
                for _ in range(3):
                    K.gemm_bf16(a, w, out, variant=v, **kw)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 5 if quick else 20
                # the reps as one captured graph: a ctypes launch costs ~20-27 us of host time, which would
                # bound the small WavLM encoder shapes (a plain loop timed QKV at 27.3 us whatever the variant)
                gph = torch.cuda.CUDAGraph()
                cs = torch.cuda.Stream()
                cs.wait_stream(torch.cuda.current_stream())
                with torch.cuda.graph(gph, stream=cs):
                    for _ in range(reps):
                        K.gemm_bf16(a, w, out, variant=v, **kw)
                torch.cuda.current_stream().wait_stream(cs)
                gph.replay()
                torch.cuda.synchronize()
                e0.record()
                gph.replay()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / reps
                outs[v] = out.float()
                ref_v = VARIANTS[0]
                d = float((outs[v] - outs[ref_v]).abs().max()) if v != ref_v else 0.0
                print(f"{name:14s} M={M:6d} N={N:5d} K={Kd:5d} v{v}: {ms*1e3:8.1f} us {2*M*N*Kd/ms/1e9:7.1f} TF/s  maxdiff_vs_first={d:.3g}",
                      flush=True)
        if "--blas" in sys.argv:  # calibration only: the vendor library (hipBLASLt) on the same shape
            if rows:  # the implicit-GEMM conv shapes: the library on a dense [M, K] operand (its best case)
                a = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                for v in VARIANTS:  # ours on the same dense operand
                    for _ in range(3):
                        K.gemm_bf16(a, w, out, variant=v)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(20):
                        K.gemm_bf16(a, w, out, variant=v)
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / 20
                    print(f"{name:14s} M={M:6d} N={N:5d} K={Kd:5d} v{v} dense: {ms*1e3:8.1f} us "
                          f"{2*M*N*Kd/ms/1e9:7.1f} TF/s", flush=True)
            wt = w.t()
            for _ in range(3):
                torch.matmul(a, wt)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                torch.matmul(a, wt)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f"{name:14s} M={M:6d} N={N:5d} K={Kd:5d} torch.matmul (hipBLASLt): {ms*1e3:8.1f} us "
                  f"{2*M*N*Kd/ms/1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
