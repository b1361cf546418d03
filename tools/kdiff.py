"""Per-kernel ms/step of two rocprofv3 kernel_stats.csv files: python tools/kdiff.py A.csv stepsA B.csv stepsB [n]"""
import csv
import sys


def load(p, steps):
    return {r["Name"][:90]: float(r["TotalDurationNs"]) / 1e6 / steps for r in csv.DictReader(open(p))}


a, b = load(sys.argv[1], float(sys.argv[2])), load(sys.argv[3], float(sys.argv[4]))
keys = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, 0), b.get(k, 0)))
for k in keys[: int(sys.argv[5]) if len(sys.argv) > 5 else 40]:
    print(f"{a.get(k, 0):7.3f} -> {b.get(k, 0):7.3f}  {b.get(k, 0) - a.get(k, 0):+7.3f}  {k}")
print(f"total {sum(a.values()):.3f} -> {sum(b.values()):.3f} ms/step")
