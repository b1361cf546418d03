"""Time the stage-2 WavLM attention backward (mer_wavlm_attention_bwd: rows + cols kernels) at the bench's
stage-2 shape (B=32 clips, L=149 frames of 3 s audio, H=12 heads, dh=64), one layer per call; with ``fwd`` the
forward (mer_wavlm_attention[_tr]) instead.
    python tools/bench_attn_bwd.py [iters] | fwd [iters]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from multimodalemotionrecognition_amd import kernels as K  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    B, L, H, dh = 32, 149, 12, 64
    D = H * dh
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
    dout = torch.randn(B * L, D, device="cuda", generator=g)
    gw = 0.1 * torch.randn(8, dh, device="cuda", generator=g)
    gb = 0.1 * torch.randn(8, device="cuda", generator=g)
    gc = 1.0 + 0.2 * torch.randn(H, device="cuda", generator=g)
    tbl = 0.5 * torch.randn(H, 2 * L - 1, device="cuda", generator=g)
    dqkv = torch.empty(B * L, 3 * D, dtype=torch.bfloat16, device="cuda")
    dxg = torch.empty(B * L, D, device="cuda")
    run = lambda: K.wavlm_attention_bwd(qkv, x, dout, gw, gb, gc, tbl, B, L, H, dh ** -0.5, dqkv, dxg)  # noqa: E731
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flop = 2.0 * B * H * L * L * dh * 5  # S, dP, dQ, dK, dV
    print(f"attention backward B={B} L={L} H={H}: {ms * 1e3:.1f} us per layer, {flop / ms / 1e9:.1f} TF/s algorithmic")


def forward_main():
    """python tools/bench_attn_bwd.py fwd [iters]: the WavLM attention forward (train mode, dropout 0.1)."""
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    B, L, H, dh = 32, 149, 12, 64
    D = H * dh
    g = torch.Generator(device="cuda").manual_seed(0)
    qkv = torch.randn(B * L, 3 * D, device="cuda", generator=g).to(torch.bfloat16)
    x = torch.randn(B * L, D, device="cuda", generator=g).to(torch.bfloat16)
    gw = 0.1 * torch.randn(8, dh, device="cuda", generator=g)
    gb = 0.1 * torch.randn(8, device="cuda", generator=g)
    gc = 1.0 + 0.2 * torch.randn(H, device="cuda", generator=g)
    tbl = 0.5 * torch.randn(H, 2 * L - 1, device="cuda", generator=g)
    out = torch.empty(B * L, D, dtype=torch.bfloat16, device="cuda")
    rng = torch.zeros(1, dtype=torch.int64, device="cuda")
    res = {}
    for p in (0.0, 0.1):
        run = lambda: K.wavlm_attention(qkv, x, gw, gb, gc, tbl, None, out, B, L, H, dh ** -0.5, drop_p=p,  # noqa: E731
                                        rng=rng if p > 0 else None, site=3)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        res[p] = e0.elapsed_time(e1) / iters * 1e3
        print(f"attention forward B={B} L={L} H={H} drop_p={p}: {res[p]:.1f} us per layer, checksum "
              f"{out.float().abs().sum().item():.6e}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "fwd":
        forward_main()
    else:
        main()
