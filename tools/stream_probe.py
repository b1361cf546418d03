"""Does work on the main stream run while the side stream is busy?  python tools/stream_probe.py
Side stream: 20 conv1-shape GEMMs (~0.34 ms each), eager or replayed from a captured graph; main stream:
a few small kernels, eager or graphed.  Prints when the main-stream work finished relative to the side
stream's start and end (events)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd import kernels as K  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    B = 32
    M, N, Kd, rows, alen = B * 4799, 512, 1536, (4799, 1024, 9599 * 512), B * 9599 * 512
    a = (torch.rand(alen, device=dev) * 2 - 1).bfloat16()
    w = (torch.rand(N, Kd, device=dev) * 2 - 1).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    side = torch.cuda.Stream(device=dev)
    small = torch.empty(1 << 20, device=dev)
    x = torch.randn(4768, 768, device=dev)
    wf = torch.randn(768, 128, device=dev)
    yo = torch.empty(4768, 128, device=dev)

    def side_work():
        for _ in range(20):
            K.gemm_bf16(a, w, out, M=M, K=Kd, rows=rows)

    def main_work():
        for _ in range(5):
            small.fill_(1.0)
            K.gemm(x, wf, yo)

    for _ in range(2):
        side_work(); main_work()
    torch.cuda.synchronize()
    gs, gm = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(cap):
        with torch.cuda.graph(gs, stream=cap):
            side_work()
        with torch.cuda.graph(gm, stream=cap):
            main_work()
    torch.cuda.synchronize()
    for side_graph in (False, True):
        for main_graph in (False, True):
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            with torch.cuda.stream(side):
                ev[0].record()
                gs.replay() if side_graph else side_work()
                ev[1].record()
            ev[2].record()
            gm.replay() if main_graph else main_work()
            ev[3].record()
            torch.cuda.synchronize()
            print(f"side {'graph' if side_graph else 'eager'} / main {'graph' if main_graph else 'eager'}: side "
                  f"{ev[0].elapsed_time(ev[1]):.2f} ms; main done at {ev[0].elapsed_time(ev[3]):.2f} ms after side start "
                  f"(main alone {ev[2].elapsed_time(ev[3]):.2f} ms span)", flush=True)


if __name__ == "__main__":
    main()
