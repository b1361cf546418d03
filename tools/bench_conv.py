"""Time conv fwd / dgrad kernel variants on the ResNet18 layers of the north-star step (256 frames of 112x112)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd import kernels as K  # noqa: E402

NF = 256
# (name, H_in, C, K, R, stride, pad)
# 112x112 frames: stem (space-to-depth 4x4 form) -> 56x56, maxpool -> layer1 28x28, layer2 14, layer3 7, layer4 4
LAYERS = [("stem s2d 4x4", 59, 16, 64, 4, 1, 0), ("layer1 3x3", 28, 64, 64, 3, 1, 1),
          ("layer2.0 3x3 s2", 28, 64, 128, 3, 2, 1), ("layer2 3x3", 14, 128, 128, 3, 1, 1),
          ("layer3.0 3x3 s2", 14, 128, 256, 3, 2, 1), ("layer3 3x3", 7, 256, 256, 3, 1, 1),
          ("layer4.0 3x3 s2", 7, 256, 512, 3, 2, 1), ("layer4 3x3", 4, 512, 512, 3, 1, 1),
          ("ds2 1x1 s2", 28, 64, 128, 1, 2, 0)]
VARIANTS = [int(v) for v in next((a.split("=")[1] for a in sys.argv if a.startswith("--variants=")), "2,4").split(",") if v]
WGRAD_V = [int(v) for v in next((a.split("=")[1] for a in sys.argv if a.startswith("--wgrad-variants=")), "1,2").split(",")
           if v]
WGRAD = "--no-wgrad" not in sys.argv
FUSED = "--fused" in sys.argv
X2 = "--x2" in sys.argv  # the fused dgrad reduces a second BN (the block-0 output of layers 2-4: bn2 + downsample BN)
ONLY = next((a.split("=")[1] for a in sys.argv if a.startswith("--layers=")), None)  # substring filter, e.g. layer1  # dgrad as in the train step: residual under a ReLU mask + the fused BN-backward sums


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    torch.manual_seed(0)
    for name, H, C, Kc, R, st, pad in LAYERS:
        if ONLY is not None and ONLY not in name:
            continue
        Ho = (H + 2 * pad - R) // st + 1
        x = (torch.rand(NF, H, H, C, device="cuda") * 2 - 1).bfloat16()
        w = torch.randn(Kc, C, R, R, device="cuda") * 0.05
        wp = torch.empty(Kc, R * R * C, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(w, wp, C, False)
        wt = torch.empty(C, R * R * Kc, device="cuda", dtype=torch.bfloat16)
        K.pack_conv_weight(w, wt, C, True)
        y = torch.empty(NF, Ho, Ho, Kc, device="cuda", dtype=torch.bfloat16)
        stats = K.bn_stats_buffer(Kc, "cuda", NF * Ho * Ho)
        dy = (torch.rand(NF, Ho, Ho, Kc, device="cuda") * 2 - 1).bfloat16()
        dx = torch.empty(NF, H, H, C, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * NF * Ho * Ho * Kc * R * R * C
        dw = torch.zeros(Kc, C, R, R, device="cuda")
        line = f"{name:16s}"
        for v in (WGRAD_V if WGRAD else ()):
            tw = timeit(lambda: K.conv_wgrad(x, dy, dw, R, R, st, pad, variant=v))
            line += f" | wgrad v{v} {tw*1e3:7.1f}us {flop/tw/1e9:6.1f}TF"
        ref_y = ref_dx = None
        fk = {}
        if FUSED and H != 59:
            res = (torch.rand_like(dx.float()) * 2 - 1).bfloat16()
            msk = (torch.rand_like(dx.float()) - 0.5).relu().bfloat16()
            xb = (torch.rand_like(dx.float()) * 2 - 1).bfloat16()
            ms = torch.stack([torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")], 1).contiguous()
            red = torch.zeros(K.bn_red_rows(NF * H * H), C, 2, device="cuda")
            fk = dict(residual=res, mask=msk, bnr=(msk, xb, ms, red))
            if X2:
                red2 = torch.zeros_like(red)
                fk["bnr"] = (msk, xb, ms, red, (torch.rand_like(dx.float()) * 2 - 1).bfloat16(), ms, red2)
        for v in VARIANTS:
            tf = timeit(lambda: K.conv_fwd(x, wp, y, stats, R, R, st, pad, variant=v))
            tb = timeit(lambda: K.conv_dgrad(dy, wt, dx, R, R, st, pad, variant=v, **fk)) if H != 59 else float("nan")
            if ref_y is None:
                ref_y, ref_dx = y.clone(), dx.clone()
            elif not (torch.equal(ref_y, y) and (H == 59 or torch.equal(ref_dx, dx))):
                line += " MISMATCH"
            line += f" | v{v} fwd {tf*1e3:7.1f}us {flop/tf/1e9:6.1f}TF dgrad {tb*1e3:7.1f}us {flop/tb/1e9:6.1f}TF"
        print(line, flush=True)


if __name__ == "__main__":
    main()
