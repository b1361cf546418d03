"""List every gfx950 kernel in the built libmer_hip.so with its private-segment (scratch) size, from the code objects'
metadata notes (objcopy the .hip_fatbin section, split its clang offload bundles, unbundle the gfx950 code
objects, llvm-readelf --notes).  Exit status 1 if any kernel uses scratch memory.

Why it matters: a kernel that uses scratch, running on one stream while a captured graph runs on another, was seen
to corrupt that graph's results on this platform: the library keeps every kernel scratch-free.
    python tools/check_scratch.py [path/to/libmer_hip.so]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
LLVM = Path("/opt/rocm/llvm/bin")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_scratch(lib: Path):
    out = {}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        fat = td / "fatbin.bin"
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", str(lib), str(td / "stripped.so")],
                       check=True, capture_output=True)
        blob = fat.read_bytes()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        for i, s in enumerate(starts):
            piece = td / f"b{i}.bin"
            piece.write_bytes(blob[s:starts[i + 1] if i + 1 < len(starts) else len(blob)])
            co = td / f"b{i}.o"
            r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={piece}", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not co.exists() or co.stat().st_size == 0:
                continue
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                                   text=True).stdout
            name = None
            for line in notes.splitlines():
                t = line.strip()
                if t.startswith(".name:"):
                    name = t.split(":", 1)[1].strip()
                elif t.startswith(".private_segment_fixed_size:") and name is not None:
                    out[name] = int(t.split(":", 1)[1])
                    name = None
    return out


def main():
    lib = Path(sys.argv[1]) if len(sys.argv) > 1 else ROOT / "multimodalemotionrecognition_amd" / "libmer_hip.so"
    ks = kernel_scratch(lib)
    bad = {k: v for k, v in ks.items() if v}
    print(f"{len(ks)} kernels, {len(bad)} with scratch")
    for k, v in sorted(bad.items()):
        print(f"  {v:5d} B  {k}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
