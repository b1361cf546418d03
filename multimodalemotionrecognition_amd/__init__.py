"""MI355X-native (gfx950 / CDNA4) fusion train / inference path for multimodal emotion recognition.

Drop-in for Wionerlol/MultimodalEmotionRecognition's ``src/models`` API on hand-written HIP
kernels (``csrc/`` -> ``libmer_hip.so``, C-ABI in ``include/mer.h``).
"""
from ._lib import LIB, MerKernelError, available, lib_path  # noqa: F401

__all__ = ["LIB", "MerKernelError", "available", "lib_path"]
