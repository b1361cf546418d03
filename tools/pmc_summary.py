"""Per-kernel averages of rocprofv3 --pmc counter CSVs: python tools/pmc_summary.py <dir with p*/> [name-filter]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if filt not in name:
            continue
        key = (name[:90], r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, ctrs in sorted(agg.items()):
    print(key)
    for c, v in sorted(ctrs.items()):
        print(f"    {c:28s} avg {sum(v) / len(v):16.1f}  (n={len(v)})")
