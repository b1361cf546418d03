"""Per-launch-shape durations of selected kernels in a rocprofv3 kernel trace (last N launches per shape):
python tools/gemm_shapes.py <kernel_trace.csv> [name-substring] [max-rows]"""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else "gemm_pipe_kernel"
by = defaultdict(list)
for r in rows:
    if pat not in r["Kernel_Name"]:
        continue
    wg = int(r["Workgroup_Size_X"])
    grid = (int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    name = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")[-70:]
    by[(name, wg, grid, int(r["LDS_Block_Size"]))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = []
for k, v in by.items():
    out.append((sum(v), k, len(v), statistics.median(v), min(v)))
for tot, k, n, med, mn in sorted(out, reverse=True)[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{tot/1e3:8.3f} ms total  n={n:4d}  med {med:8.1f}us  min {mn:8.1f}us  wg={k[1]} grid={k[2]} lds={k[3]}  {k[0]}")
