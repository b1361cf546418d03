"""Phase timing of the pipelined bf16 GEMM (csrc/gemm_bf16.hip gemm_pipe_kernel): builds
multimodalemotionrecognition_amd/libmer_hip_gt.so (the kernel library with -DMER_GEMM_TIMING, see GT() there), runs
the WavLM encoder shapes of the B=32 step through it and prints the median over workgroups of each phase (us, wall
clock): prologue (kernel entry -> first K-tile published), K loop, epilogue; and the kernel span.
    python tools/gemm_phases.py build      (here: hipcc, no GPU)
    python tools/gemm_phases.py run [--variants=18,9] [--resid] [--act=gelu] [--conv1] [--hot]   (GPU box)"""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodalemotionrecognition_amd"
GT_LIB = PKG / "libmer_hip_gt.so"


def build():
    csrc = PKG / "csrc"
    out = csrc / "build" / "gt"
    out.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-DMER_GEMM_TIMING", f"-I{ROOT / 'include'}",
             "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    o = out / "gemm_bf16.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", str(csrc / "gemm_bf16.hip"), "-o", str(o)])
    objs = [str(p) for p in sorted((csrc / "build").glob("*.o")) if p.name != "gemm_bf16.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(o), *objs, "-o",
                           str(GT_LIB)])


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import _lib
    _lib._LIB_PATH = GT_LIB  # the instrumented library (this tool only)
    from multimodalemotionrecognition_amd import kernels as K
    variants = [int(v) for v in next((a.split("=")[1] for a in sys.argv if a.startswith("--variants=")),
                                     "18").split(",")]
    resid = "--resid" in sys.argv
    act = next((a.split("=")[1] for a in sys.argv if a.startswith("--act=")), "none")
    warm = 2000 if "--hot" in sys.argv else 3  # --hot: ~2 s of back-to-back launches first (the clock under load)
    M = 32 * 149
    shapes = {"qkv": (2304, 768), "ffn1": (3072, 768), "ffn2": (768, 3072), "out_proj": (768, 768)}
    if "--conv1" in sys.argv:  # the feature extractor's conv1 as an implicit GEMM (rows mode, tools/bench_gemm.py)
        shapes = {"conv1": (512, 1536)}
    tick_us = 0.01
    for name, (N, Kd) in shapes.items():
        kw = {}
        if name == "conv1":
            Mr = 32 * 4799
            a = (torch.rand(32 * 9599 * 512, device="cuda") * 2 - 1).bfloat16()
            kw = dict(M=Mr, K=Kd, rows=(4799, 1024, 9599 * 512))
        else:
            Mr = M
            a = (torch.rand(M, Kd, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(N, Kd, device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(Mr, N, device="cuda", dtype=torch.bfloat16)
        r = (torch.rand(Mr, N, device="cuda") * 2 - 1).bfloat16() if resid else None
        bias = torch.rand(N, device="cuda")
        for v in variants:
            for _ in range(warm):
                K.gemm_bf16(a, w, out, bias=bias, residual=r, act=act, variant=v, **kw)
            torch.cuda.synchronize()
            assert _lib.LIB._dll.mer_gt_reset() == 0
            K.gemm_bf16(a, w, out, bias=bias, residual=r, act=act, variant=v, **kw)
            torch.cuda.synchronize()
            t = np.zeros((1024, 8), dtype=np.int64)
            assert _lib.LIB._dll.mer_gt_read(ctypes.c_void_p(t.ctypes.data)) == 0
            used = [b for b in range(1024) if t[b, 0] and t[b, 3]]
            ph = [np.median([(t[b, k] - t[b, k - 1]) * tick_us for b in used]) for k in (1, 2, 3)]
            # slots 5 / 6: s_memtime (shader cycles) at the K loop's start / end: the in-kernel clock over the loop and
            # the loop's MFMA-pipe occupancy at that clock (256^2 tiles: 4 waves per SIMD x 32 MFMAs x 16 cycles per
            # 64-deep K-tile)
            cyc = [t[b, 6] - t[b, 5] for b in used if t[b, 5] and t[b, 6]]
            ghz = np.median([(t[b, 6] - t[b, 5]) / ((t[b, 2] - t[b, 1]) * 10.0) for b in used if t[b, 5] and t[b, 6]]) \
                if cyc else float("nan")
            per_kt = {13: 2048, 18: 2048, 21: 2048}.get(v)
            occ = (Kd // 64) * per_kt / np.median(cyc) if (cyc and per_kt) else float("nan")
            # slot 4: after the epilogue's opening barrier (waits for the slowest wave's last MFMAs)
            sync = np.median([(t[b, 4] - t[b, 2]) * tick_us for b in used]) if all(t[b, 4] for b in used) else float("nan")
            tot = [(t[b, 3] - t[b, 0]) * tick_us for b in used]
            st = [(t[b, 0] - min(t[u, 0] for u in used)) * tick_us for b in used]
            span = (max(t[b, 3] for b in used) - min(t[b, 0] for b in used)) * tick_us
            print(f"{name:9s} N={N:5d} K={Kd:5d} v{v}{' resid' if resid else ''}{' ' + act if act != 'none' else ''}: blocks {len(used):4d}  prologue "
                  f"{ph[0]:6.2f}  K loop {ph[1]:6.2f}  epilogue {ph[2]:6.2f} (barrier {sync:5.2f}) | block {np.median(tot):6.2f} max "
                  f"{max(tot):6.2f}  last start {max(st):6.2f}  span {span:6.2f} us | loop clock {ghz:4.2f} GHz, MFMA "
                  f"occupancy {occ:4.2f}", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
