"""Phase timing of conv_pipe_kernel (csrc/conv.hip, CTP() stamps of a -DMER_CONV_TIMING build, see halo_phases.py):
per launch, the median over workgroups of prologue (address setup + first DMAs), K loop, split-K exchange, epilogue,
and the launch span; stride-2 input gradients per parity class.  Shapes of the B=32 step (256 frames of 112x112).
    python tools/pipe_phases.py build      (here: hipcc, no GPU)
    python tools/pipe_phases.py run [variants, e.g. 2,7,8]   (GPU box)"""
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import halo_phases  # noqa: E402

NF = 256
# (name, H_in, C, K, stride)
SHAPES = [("layer2 3x3", 14, 128, 128, 1), ("layer3.0 s2", 14, 128, 256, 2), ("layer3 3x3", 7, 256, 256, 1),
          ("layer4.0 s2", 7, 256, 512, 2), ("layer4 3x3", 4, 512, 512, 1)]


def run(variants):
    import numpy as np
    import torch
    sys.path.insert(0, str(ROOT))
    from multimodalemotionrecognition_amd import _lib
    _lib._LIB_PATH = halo_phases.CT_LIB
    from multimodalemotionrecognition_amd import kernels as K
    tick_us = 0.01  # wall_clock64: 100 MHz
    torch.manual_seed(0)
    for name, H, C, Kc, st in SHAPES:
        Ho = (H + 2 - 3) // st + 1
        x = (torch.rand(NF, H, H, C, device="cuda") * 2 - 1).bfloat16()
        w = torch.randn(Kc, C, 3, 3, device="cuda") * 0.05
        wp = torch.empty(Kc, 9 * C, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(w, wp, C, False)
        wt = torch.empty(C, 9 * Kc, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(w, wt, C, True)
        y = torch.empty(NF, Ho, Ho, Kc, device="cuda", dtype=torch.bfloat16)
        stats = K.bn_stats_buffer(Kc, "cuda", NF * Ho * Ho)
        dy = (torch.rand(NF, Ho, Ho, Kc, device="cuda") * 2 - 1).bfloat16()
        dx = torch.empty(NF, H, H, C, device="cuda", dtype=torch.bfloat16)
        res = (torch.rand_like(dx.float()) * 2 - 1).bfloat16()
        msk = (torch.rand_like(dx.float()) - 0.5).relu().bfloat16()
        ms = torch.stack([torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")], 1).contiguous()
        red = torch.zeros(K.bn_red_rows(NF * H * H), C, 2, device="cuda")
        for v in variants:
            runs = {"fwd": lambda: K.conv_fwd(x, wp, y, stats, 3, 3, st, 1, variant=v),
                    "dgrad": lambda: K.conv_dgrad(dy, wt, dx, 3, 3, st, 1, residual=res, mask=msk, variant=v,
                                                  bnr=(msk, x, ms, red))}
            for kind, fn in runs.items():
                for _ in range(4):
                    fn()
                torch.cuda.synchronize()
                assert _lib.LIB._dll.mer_ctp_reset() == 0
                assert _lib.LIB._dll.mer_ct_reset() == 0
                fn()
                torch.cuda.synchronize()
                t = np.zeros((4096, 8), dtype=np.int64)
                assert _lib.LIB._dll.mer_ctp_read(ctypes.c_void_p(t.ctypes.data)) == 0
                used = np.array([b for b in range(4096) if t[b, 0] != 0 and t[b, 4] != 0])
                if not len(used):
                    print(f"{name:12s} {kind:5s} v{v}: no stamps")
                    continue
                tt = t[used].astype(np.float64)
                t0, t1 = tt[:, 0].min(), tt[:, 4].max()
                ph = [np.median(tt[:, k + 1] - tt[:, k]) * tick_us for k in range(4)]
                tot = np.median(tt[:, 4] - tt[:, 0]) * tick_us
                starts = np.sort(tt[:, 0] - t0) * tick_us
                line = (f"{name:12s} {kind:5s} v{v}: WGs {len(used):4d} span {(t1 - t0) * tick_us:6.2f} | per WG: "
                        f"pro {ph[0]:5.2f} K {ph[1]:6.2f} xchg {ph[2]:5.2f} epi {ph[3]:5.2f} tot {tot:6.2f} | "
                        f"last start {starts[-1]:6.2f}")
                c = np.zeros((512, 64), dtype=np.int64)
                assert _lib.LIB._dll.mer_ct_read(ctypes.c_void_p(c.ctypes.data)) == 0
                sel = [i for i, b in enumerate(used) if b < 512 and c[b, 10] and c[b, 11] and c[b, 12]]
                if sel and st == 1:  # epilogue detail: passes | cross-lane / cross-wave reductions + row stores | flush
                    b = used[sel]
                    p1 = np.median(c[b, 10] - tt[sel, 3]) * tick_us
                    p2 = np.median(c[b, 11] - c[b, 10]) * tick_us
                    p3 = np.median(c[b, 12] - c[b, 11]) * tick_us
                    line += f" | epi: passes {p1:5.2f} reduce {p2:5.2f} flush {p3:5.2f}"
                    if kind == "dgrad" and all(c[b, 13]) and all(c[b, 14]):  # reduce = xor tree | barrier | rest
                        x1 = np.median(c[b, 13] - c[b, 10]) * tick_us
                        x2 = np.median(c[b, 14] - c[b, 13]) * tick_us
                        x3 = np.median(c[b, 11] - c[b, 14]) * tick_us
                        line += f" (xor {x1:5.2f} barrier {x2:5.2f} meet+store {x3:5.2f})"
                if st == 2 and kind == "dgrad":
                    # grid.y = parity class slot (3 - class); linear id = y * gridDim.x + x
                    gx = (max(used) // 4) + 1 if False else None
                    nxm = int(np.ceil((used.max() + 1) / 4))
                    for y_ in range(4):
                        sel = (used // nxm) == y_
                        if sel.any():
                            line += f" | cls{3 - y_}: K {np.median(tt[sel, 2] - tt[sel, 1]) * tick_us:5.2f}"
                print(line, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        halo_phases.build()
    else:
        run([int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "2,7,8").split(",")])
