"""Phase timing of the layer1 halo conv (csrc/conv.hip conv3x3_halo_kernel): builds
multimodalemotionrecognition_amd/libmer_hip_ct.so (the kernel library with -DMER_CONV_TIMING, see CT() in conv.hip),
runs the stem (space-to-depth form) and the layer1 forward and input-gradient shapes of the B=32 step (256 frames, 28x28x64) through it and prints the
median over workgroups of each phase (us, wall clock): prologue (weights + first halo), then per tile: K loop,
halo wait + barrier, epilogue, end barrier.
    python tools/halo_phases.py build      (here: hipcc, no GPU)
    python tools/halo_phases.py run        (GPU box)"""
import ctypes
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodalemotionrecognition_amd"
CT_LIB = PKG / "libmer_hip_ct.so"


def build():
    csrc = PKG / "csrc"
    out = csrc / "build" / "ct"
    out.mkdir(parents=True, exist_ok=True)
    flags = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-DMER_CONV_TIMING", f"-I{ROOT / 'include'}",
             "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    o = out / "conv.o"
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, "-c", str(csrc / "conv.hip"), "-o", str(o)])
    objs = [str(p) for p in sorted((csrc / "build").glob("*.o")) if p.name != "conv.o"]
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", str(o), *objs, "-o",
                           str(CT_LIB)])


def run():
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import _lib
    _lib._LIB_PATH = CT_LIB  # the instrumented library (this tool only)
    from multimodalemotionrecognition_amd import kernels as K
    NF, H, C = 256, 28, 64
    x = (torch.rand(NF, H, H, C, device="cuda") * 2 - 1).bfloat16()
    w = torch.randn(C, C, 3, 3, device="cuda") * 0.05
    wp = torch.empty(C, 9 * C, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(w, wp, C, False)
    y = torch.empty_like(x)
    st = K.bn_stats_buffer(C, "cuda", NF * H * H)
    res = (torch.rand_like(x.float()) * 2 - 1).bfloat16()
    msk = (torch.rand_like(x.float()) - 0.5).relu().bfloat16()
    ms = torch.stack([torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")], 1).contiguous()
    red = torch.zeros(K.bn_red_rows(NF * H * H), C, 2, device="cuda")
    xs = (torch.rand(NF, 59, 59, 16, device="cuda") * 2 - 1).bfloat16()
    ws = torch.randn(64, 16, 4, 4, device="cuda") * 0.05
    wsp = torch.empty(64, 256, device="cuda", dtype=torch.bfloat16)
    K.pack_conv_weight(ws, wsp, 16, False)
    ys = torch.empty(NF, 56, 56, 64, device="cuda", dtype=torch.bfloat16)
    sts = K.bn_stats_buffer(64, "cuda", NF * 56 * 56)
    runs = {"stem": lambda: K.conv_fwd(xs, wsp, ys, sts, 4, 4, 1, 0, variant=6),
            "fwd": lambda: K.conv_fwd(x, wp, y, st, 3, 3, 1, 1, variant=6),
            "dgrad": lambda: K.conv_dgrad(x, wp, y, 3, 3, 1, 1, residual=res, mask=msk, variant=6,
                                          bnr=(msk, x, ms, red))}
    tick_us = 0.01  # wall_clock64: 100 MHz
    for name, fn in runs.items():
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
        assert _lib.LIB._dll.mer_ct_reset() == 0
        fn()
        torch.cuda.synchronize()
        t = np.zeros((512, 64), dtype=np.int64)
        assert _lib.LIB._dll.mer_ct_read(ctypes.c_void_p(t.ctypes.data)) == 0
        used = [b for b in range(512) if t[b, 0] != 0]
        t0 = min(t[b, 0] for b in used)
        pro = np.median([(t[b, 1] - t[b, 0]) * tick_us for b in used])
        line = f"{name:6s} WGs {len(used)} prologue {pro:5.2f}"
        for it in range(11):
            ks = [2 + 5 * it + k for k in range(5)]
            have = [b for b in used if all(t[b, k] for k in ks)]
            if not have:
                break
            ph = [np.median([(t[b, ks[k + 1]] - t[b, ks[k]]) * tick_us for b in have]) for k in range(4)]
            line += f" | t{it}: K {ph[0]:4.2f} wait {ph[1]:4.2f} epi {ph[2]:4.2f} bar {ph[3]:4.2f}"
        e = [b for b in used if t[b, 60] and t[b, 61] and t[b, 62] and t[b, 9]]
        if e:  # inside tile 1's epilogue (slot 9 = its start): staging passes, reductions, stores issued
            line += (f" | epi(t1): passes {np.median([(t[b, 60] - t[b, 9]) * tick_us for b in e]):4.2f} reduce "
                     f"{np.median([(t[b, 61] - t[b, 60]) * tick_us for b in e]):4.2f} stores "
                     f"{np.median([(t[b, 62] - t[b, 61]) * tick_us for b in e]):4.2f}")
        end = max(max(t[b, k] for k in range(60) if t[b, k]) for b in used)
        print(line + f" | span {(end - t0) * tick_us:6.2f} us", flush=True)


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
