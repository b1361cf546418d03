"""VGPR / AGPR / SGPR / LDS / scratch of every kernel in the built libmer_hip.so matching a substring (code-object
metadata notes): the occupancy side of a kernel's time.
    python tools/kernel_regs.py [substring] [path/to/lib.so]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from check_codeobj import LLVM, ROOT, _code_objects  # noqa: E402


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    lib = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "multimodalemotionrecognition_amd" / "libmer_hip.so"
    keys = (".vgpr_count", ".agpr_count", ".sgpr_count", ".group_segment_fixed_size", ".private_segment_fixed_size",
            ".max_flat_workgroup_size")
    with tempfile.TemporaryDirectory() as td:
        for co in _code_objects(lib, Path(td)):
            notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(co)], capture_output=True,
                                   text=True).stdout
            cur = {}
            for line in notes.splitlines():
                t = line.strip().lstrip("- ")
                for k in keys + (".name",):
                    if t.startswith(k + ":"):
                        cur[k] = t.split(":", 1)[1].strip()
                if ".name" in cur and all(k in cur for k in keys):
                    if pat in cur[".name"]:
                        dem = subprocess.run(["c++filt"], input=cur[".name"], capture_output=True,
                                             text=True).stdout.strip()
                        print(f"v{cur['.vgpr_count']:>4s} a{cur['.agpr_count']:>4s} s{cur['.sgpr_count']:>4s} "
                              f"lds{cur['.group_segment_fixed_size']:>6s} scr{cur['.private_segment_fixed_size']:>4s} "
                              f"wg{cur['.max_flat_workgroup_size']:>5s}  {re.sub(r'(anonymous namespace)::', '', dem)[:150]}")
                    cur = {}


if __name__ == "__main__":
    main()
