"""Do the frozen WavLM (side stream) and the ResNet18 trunk (main stream) actually overlap?
python tools/overlap_probe.py  -> device time of each alone and of both issued together."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
from multimodalemotionrecognition_amd.train import build_model  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = build_model(8, "xattn", pretrained_video=False, use_wavlm=True).to(dev)
    model.train()
    video, audio, labels = bench.synthetic_batch(dev, 1)
    side = torch.cuda.Stream(device=dev)
    b, t = video.shape[:2]
    v_in = video.reshape(b * t, *video.shape[2:])

    def wav():
        with torch.no_grad():
            return model.audio_model.encode_sequence(audio)

    def trunk():
        with torch.no_grad():
            return model.video_model.backbone(v_in)

    def both():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            wav()
        trunk()
        cur.wait_stream(side)

    def both_side_trunk():  # trunk on the side stream, WavLM on main
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            trunk()
        wav()
        cur.wait_stream(side)

    print(f"wavlm alone {timed(wav):.3f} ms, trunk fwd alone {timed(trunk):.3f} ms, "
          f"both (wavlm side) {timed(both):.3f} ms, both (trunk side) {timed(both_side_trunk):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
