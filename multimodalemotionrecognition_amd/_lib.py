"""ctypes binding of the C-ABI kernel library (``include/mer.h`` -> ``libmer_hip.so``).

The library is built in-tree (``__graft_entry__.build()`` / ``make -C
multimodalemotionrecognition_amd/csrc``) so it travels with the repo snapshot.
There is no fallback: if the shared object is missing or a kernel returns a
non-zero ``hipError_t``, a ``MerKernelError`` is raised.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

# MER_HIP_LIB: load another build of the same ABI instead (A/B timing of a kernel change in one process tree)
_LIB_PATH = Path(os.environ.get("MER_HIP_LIB") or Path(__file__).resolve().parent / "libmer_hip.so")

_HEADER = Path(__file__).resolve().parents[1] / "include" / "mer.h"


def parse_header(path: Path = _HEADER):
    """Parse ``int mer_xxx(...);`` prototypes of include/mer.h into ctypes argument codes.

    The header is the single source of truth for the ABI (the .hip sources include it, so the
    compiler checks definitions against it); codes: i=int32 l=int64 f=float u=uint64 p=pointer.
    """
    text = re.sub(r"/\*.*?\*/", " ", path.read_text(), flags=re.S)
    sigs = {}
    for m in re.finditer(r"\bint\s+(mer_\w+)\s*\(([^)]*)\)\s*;", text):
        codes = []
        for arg in m.group(2).split(","):
            arg = " ".join(arg.split())
            if not arg or arg == "void":
                continue
            if "*" in arg:
                codes.append("p")
            elif arg.startswith("unsigned long long"):
                codes.append("u")
            elif arg.startswith("long"):
                codes.append("l")
            elif arg.startswith("float"):
                codes.append("f")
            elif arg.startswith("int"):
                codes.append("i")
            else:
                raise ValueError(f"unsupported C type in {m.group(1)}: {arg}")
        sigs[m.group(1)] = "".join(codes)
    return sigs


_CT = {"i": ctypes.c_int, "l": ctypes.c_long, "f": ctypes.c_float, "u": ctypes.c_ulonglong, "p": ctypes.c_void_p}


class MerKernelError(RuntimeError):
    pass


class _Lib:
    def __init__(self) -> None:
        self._dll = None
        self._fns = {}

    def load(self):
        if self._dll is None:
            if not _LIB_PATH.exists():
                raise MerKernelError(
                    f"HIP kernel library not built: {_LIB_PATH} is missing. Run "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)."
                )
            self._dll = ctypes.CDLL(str(_LIB_PATH))
            for name, sig in parse_header().items():
                fn = getattr(self._dll, name)
                fn.argtypes = [_CT[c] for c in sig]
                fn.restype = ctypes.c_int
                self._fns[name] = fn
        return self

    def symbols(self):
        self.load()
        return list(self._fns)

    def __call__(self, name: str, *args):
        self.load()
        rc = self._fns[name](*args)
        if rc != 0:
            raise MerKernelError(f"{name} failed with hipError_t {rc}")

    def call_int(self, name: str, *args) -> int:
        """An entry point whose int result is a value (e.g. mer_conv_fwd_rows), not a hipError_t."""
        self.load()
        return self._fns[name](*args)


LIB = _Lib()


def lib_path() -> Path:
    return _LIB_PATH


def available() -> bool:
    return _LIB_PATH.exists() and os.access(_LIB_PATH, os.R_OK)
