"""Per-kernel HBM traffic of a whole bench.py run from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate
runs, tools/scratch-style script: rocprofv3 --pmc FETCH_SIZE -d <dir>/fetch ... ; --pmc WRITE_SIZE -d <dir>/write ...):
    python tools/pmc_step_traffic.py <dir> [top_n]
FETCH_SIZE (KB) is doubled (gfx950 reports half of a 16-B/lane streaming read, MI355X_MICROARCH.md 'HBM'),
WRITE_SIZE (KB) is exact.  Prints, per kernel name, launches and the average MB fetched / written per launch, sorted
by total traffic: a kernel far above its algorithmic bytes re-reads (the first thing to fix)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40


def load(sub, name):
    acc = defaultdict(list)
    for f in glob.glob(f"{root}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name:
                acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


fetch, write = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
rows = []
for k in set(fetch) | set(write):
    f, w = fetch.get(k, []), write.get(k, [])
    fa = 2 * sum(f) / len(f) / 1024 if f else 0.0  # MB per launch
    wa = sum(w) / len(w) / 1024 if w else 0.0
    n = max(len(f), len(w))
    rows.append((n * (fa + wa), n, fa, wa, k))
rows.sort(reverse=True)
print(f"{'total MB':>10s} {'n':>5s} {'fetch MB':>9s} {'write MB':>9s}  kernel")
for tot, n, fa, wa, k in rows[:top]:
    print(f"{tot:10.1f} {n:5d} {fa:9.2f} {wa:9.2f}  {k[:110]}")
