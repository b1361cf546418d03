"""The ResNet18 trunk ALONE (VideoNet.backbone, video.py:21-23) at the north-star step's shape -- 256 frames of
112x112 (B=32 clips x 8) -- forward + backward + FusedAdam, on one stream with nothing beside it: the serialized
per-kernel trace tools/trunk_table.py turns into the per-conv roofline table (the production step runs the frozen
WavLM on a second stream, whose kernels share the CUs and stretch every duration in a two-stream trace).
    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- python tools/trunk_serial.py [steps]
    python tools/trunk_table.py DIR/.../run_kernel_trace.csv > profiles/<round>/trunk_table_serial.txt"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from multimodalemotionrecognition_amd.optim import FusedAdam  # noqa: E402
from multimodalemotionrecognition_amd.train import build_model  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.manual_seed(0)
    m = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).cuda().train()
    bb = m.video_model.backbone
    params = [q for q in bb.parameters() if q.requires_grad]
    opt = FusedAdam(params, lr=1e-3, weight_decay=1e-4)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(256, 3, 112, 112, device="cuda", generator=g)
    dy = torch.randn(256, 512, 1, 1, device="cuda", generator=g)
    for _ in range(steps):
        opt.zero_grad()
        feat = bb(x)
        feat.backward(dy)
        opt.step()
    torch.cuda.synchronize()
    print(f"trunk alone: {steps} fwd+bwd+Adam steps done")


if __name__ == "__main__":
    main()
