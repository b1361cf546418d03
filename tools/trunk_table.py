"""Per-layer table of the ResNet18 trunk (fwd conv, dgrad, wgrad) from a rocprofv3 kernel trace of bench.py:
layer, GEMM shape (M x N x K), us per launch, TF/s -- one steady-state step, launches labelled by the trunk's
fixed launch order (video.py: forward stem + per block conv1, conv2, [downsample]; backward per block in
reverse: wgrad conv2, dgrad conv2, wgrad conv1, [wgrad ds], dgrad conv1 (with the downsample's dgrad fused in,
video.FUSED_DS_DGRAD; MER_TRUNK_UNFUSED_DS=1 for traces of the two-launch form); stem wgrad last).
    python tools/trunk_table.py <run_kernel_trace.csv> [train_steps_in_trace] > profiles/<round>/trunk_table.txt
Each launch also gets its roofline: attainable = min(dense bf16 MFMA peak, FLOPs / algorithmic bytes x 8 TB/s) with
the algorithmic bytes = the bf16 A source read once + the bf16 weights + the bf16 output (wgrad: both activations +
the fp32 weight gradient), and frac = achieved / attainable.  tools/trunk_serial.py makes a serialized
(single-stream, trunk-only) trace for this table."""
import csv
import sys as _sys
from pathlib import Path as _Path

_sys.path.insert(0, str(_Path(__file__).resolve().parent))
from pmc_head import kernel_key  # noqa: E402  (demangled-name key that keeps anonymous-namespace kernels)
import os
import sys

NIMG, H = 256, 112  # B=32 clips x 8 frames, 112x112
PEAK_TF, HBM_TBS = 2500.0, 8.0  # MI355X dense bf16 MFMA, HBM3E (MI355X_MICROARCH.md)


def conv_bytes(kind, c):
    """Algorithmic HBM bytes of one launch: (name, M, N, K) with K = taps * Cin; bf16 activations."""
    _, M, N, Kr = c
    name = c[0]
    taps = 49 if name.startswith("stem") else (1 if "downsample" in name else 9)
    cin = Kr // taps
    stride = 2 if ("downsample" in name or name.startswith("stem") or ".0.conv1" in name and not name.startswith(
        "layer1")) else 1
    m_in = M * stride * stride  # input pixels (the stem: 3 channels of 112^2 per output 56^2)
    if kind == "wgrad":
        return 2 * m_in * cin + 2 * M * N + 4 * N * Kr
    return 2 * m_in * cin + 2 * N * Kr + 2 * M * N


def roof(flop, byt, us):
    ach = flop / us / 1e6
    att = min(PEAK_TF, flop / byt * HBM_TBS)
    return ach, att, ach / att


def trunk_convs():
    """(name, M, N, K) of every conv in forward order (torchvision ResNet18 at 112x112; the stem as 7x7/s2)."""
    convs = [("stem 7x7/2", NIMG * 56 * 56, 64, 3 * 49)]
    hw, cin = 28, 64
    for li, cout in enumerate((64, 128, 256, 512)):
        for bi in range(2):
            s = 2 if (bi == 0 and li > 0) else 1
            ho = (hw + 2 - 3) // s + 1
            convs.append((f"layer{li + 1}.{bi}.conv1", NIMG * ho * ho, cout, cin * 9))
            convs.append((f"layer{li + 1}.{bi}.conv2", NIMG * ho * ho, cout, cout * 9))
            if bi == 0 and li > 0:
                convs.append((f"layer{li + 1}.{bi}.downsample", NIMG * ho * ho, cout, cin))
            hw, cin = ho, cout
    return convs


FUSED_DS = os.environ.get("MER_TRUNK_UNFUSED_DS", "0") != "1"


def backward_order(convs):
    """(kind, conv, extra FLOPs) in the backward launch order."""
    blocks = {}
    for c in convs[1:]:
        blocks.setdefault(c[0].rsplit(".", 1)[0], {})[c[0].rsplit(".", 1)[1]] = c
    order = []
    for name in reversed(list(blocks)):
        b = blocks[name]
        order += [("wgrad", b["conv2"], 0.0), ("dgrad", b["conv2"], 0.0), ("wgrad", b["conv1"], 0.0)]
        if "downsample" in b:
            ds, c1 = b["downsample"], b["conv1"]
            order.append(("wgrad", ds, 0.0))
            if FUSED_DS:  # one launch: conv1's dgrad with the downsample's as an extra K segment (FLOPs of both)
                order.append(("dgrad", (c1[0] + "+ds",) + c1[1:], 2.0 * ds[1] * ds[2] * ds[3]))
                continue
            order.append(("dgrad", ds, 0.0))
        order.append(("dgrad", b["conv1"], 0.0))
    order.append(("wgrad", convs[0], 0.0))
    return order


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("adam_kernel")]
    per = max(1, round(len(adam) / int(sys.argv[2]))) if len(sys.argv) > 2 else 1
    ends = adam[per - 1::per]
    a, b = ends[-3], ends[-2]  # one steady-state step
    win = rows[a + 1:b + 1]
    convs = trunk_convs()
    fwd = [r for r in win if "conv_pipe_kernel<false" in r["Kernel_Name"].replace(" ", "")
           or "conv_halo_kernel<false" in r["Kernel_Name"].replace(" ", "")]
    bwd = [r for r in win if "conv_pipe_kernel<true" in r["Kernel_Name"].replace(" ", "")
           or "conv_halo_kernel<true" in r["Kernel_Name"].replace(" ", "")
           or "(anonymousnamespace)::wgrad_kernel<" in r["Kernel_Name"].replace(" ", "")
           or "(anonymousnamespace)::wgrad_pipe_kernel<" in r["Kernel_Name"].replace(" ", "")]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    print(f"{'layer':26s} {'pass':6s} {'M x N x K':>22s} {'us':>8s} {'TF/s':>7s} {'attain':>7s} {'frac':>6s}  kernel")
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    flops = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for c, r in zip(convs, fwd):
        us = dur(r)
        f = 2.0 * c[1] * c[2] * c[3]
        tot["fwd"] += us
        flops["fwd"] += f
        _, att, fr = roof(f, conv_bytes("fwd", c), us)
        print(f"{c[0]:26s} {'fwd':6s} {c[1]:>9d}x{c[2]:>4d}x{c[3]:>5d} {us:8.1f} {f / us / 1e6:7.1f} {att:7.0f} {fr:6.3f}  "
              f"{r['Kernel_Name'][:60]}")
    for (kind, c, extra), r in zip(backward_order(convs), bwd):
        us = dur(r)
        f = 2.0 * c[1] * c[2] * c[3] + extra
        tot[kind] += us
        flops[kind] += f
        _, att, fr = roof(f, conv_bytes(kind, c), us)
        print(f"{c[0]:26s} {kind:6s} {c[1]:>9d}x{c[2]:>4d}x{c[3]:>5d} {us:8.1f} {f / us / 1e6:7.1f} {att:7.0f} {fr:6.3f}  "
              f"{r['Kernel_Name'][:60]}")
    if len(fwd) != len(convs) or len(bwd) != len(backward_order(convs)):
        print(f"# WARNING: matched {len(fwd)} fwd / {len(bwd)} bwd launches, expected {len(convs)} / "
              f"{len(backward_order(convs))}")
    for k in tot:
        print(f"# {k}: {tot[k]:.1f} us, {flops[k] / 1e9:.1f} GFLOP, {flops[k] / tot[k] / 1e6:.1f} TF/s")
    other = {}
    for r in win:
        n = r["Kernel_Name"]
        if any(s in n for s in ("bn_", "wgrad_reduce", "wgrad_scatter", "wgrad_fold", "pack_w", "pack_input", "stem_",
                                "maxpool", "avgpool", "partials_sum")):
            key = kernel_key(n)[:60]
            other[key] = other.get(key, 0.0) + dur(r)
    print(f"# conv total {sum(tot.values()):.1f} us; BN / pack / weight-gradient fold / pool kernels "
          f"{sum(other.values()):.1f} us; serialized trunk {sum(tot.values()) + sum(other.values()):.1f} us:")
    for k, v in sorted(other.items(), key=lambda kv: -kv[1]):
        print(f"#   {v:8.1f} us  {k}")


if __name__ == "__main__":
    main()
