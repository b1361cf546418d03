"""Ad-hoc timing of the HIP path pieces on one GPU (random init, synthetic clips)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, n=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    from multimodalemotionrecognition_amd.wavlm_audio import WavLMBackbone
    from multimodalemotionrecognition_amd import kernels as K
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    m = WavLMBackbone().cuda()
    wav = (0.1 * torch.randn(B, 48000)).clamp(-1, 1).cuda()
    ms = timeit(lambda: m.forward_hip(wav))
    print(f"wavlm fwd B={B}: {ms:.2f} ms  ({42.4e9 * B / (ms * 1e-3) / 1e12:.1f} TFLOP/s algorithmic)")
    for (M, N, Kd) in [(4768, 2304, 768), (4768, 3072, 768), (4768, 768, 3072), (153568, 512, 1536)]:
        a = torch.randn(M, Kd, device="cuda").bfloat16()
        w = torch.randn(N, Kd, device="cuda").bfloat16()
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ms = timeit(lambda: K.gemm_bf16(a, w, o), n=20)
        print(f"gemm_bf16 {M}x{N}x{Kd}: {ms:.3f} ms {2 * M * N * Kd / (ms * 1e-3) / 1e12:.1f} TFLOP/s")


if __name__ == "__main__":
    main()
