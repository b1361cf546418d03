"""MI355X-native (gfx950 / CDNA4) fusion train / inference path for multimodal emotion recognition.

Drop-in for Wionerlol/MultimodalEmotionRecognition's ``src/models`` API on hand-written HIP
kernels (``csrc/`` -> ``libmer_hip.so``, C-ABI in ``include/mer.h``).
"""
from ._lib import LIB, MerKernelError, available, lib_path  # noqa: F401


def __getattr__(name):
    # reference-named model classes, imported lazily (src/models/{fusion,video,wavlm_audio}.py)
    if name == "FusionModel":
        from .fusion import FusionModel
        return FusionModel
    if name == "VideoNet":
        from .video import VideoNet
        return VideoNet
    if name == "WavLMAudioEncoder":
        from .wavlm_audio import WavLMAudioEncoder
        return WavLMAudioEncoder
    raise AttributeError(name)


__all__ = ["LIB", "MerKernelError", "available", "lib_path", "FusionModel", "VideoNet", "WavLMAudioEncoder"]
