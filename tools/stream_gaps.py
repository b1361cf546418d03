"""Per-stream busy time and the largest idle gaps of one steady-state step in a rocprofv3 kernel trace:
python tools/stream_gaps.py <run_kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
adam = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("adam_kernel")]
ends = adam[2::3]
a, b = ends[-3], ends[-2]
t0 = int(rows[a]["End_Timestamp"])
st = [((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3, r["Stream_Id"], r["Kernel_Name"][:60])
      for r in rows[a + 1:b + 1]]
print(f"step span {st[-1][1]:.0f} us")
by = defaultdict(list)
for x in st:
    by[x[2]].append(x)
for s, xs in by.items():
    busy = sum(e - b_ for b_, e, _, _ in xs)
    print(f"stream {s}: {len(xs)} kernels, busy {busy:.0f} us, first {xs[0][0]:.0f} last {xs[-1][1]:.0f}")
    for i in range(len(xs) - 1):
        g = xs[i + 1][0] - xs[i][1]
        if g > 100:
            print(f"   gap {g:.0f} us at {xs[i][1]:.0f} after {xs[i][3]} before {xs[i + 1][3]}")
