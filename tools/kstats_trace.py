"""Steady-state per-step kernel time from a rocprofv3 kernel_trace.csv of bench.py: steps are delimited
by the optimizer's last adam_kernel launch of each step, setup/warm-up windows are dropped.
    python tools/kstats_trace.py <run_kernel_trace.csv> [top] [train_steps_in_trace]
(train_steps_in_trace = warmup + steps + probe steps + 2 of the bench run; it sets the adam launches per step,
default 1 -- FusedAdam launches one adam_kernel per run of equal step counts, one per step in the bench)"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
adam = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("adam_kernel")]
per = max(1, round(len(adam) / int(sys.argv[3]))) if len(sys.argv) > 3 else 1
ends = adam[per - 1::per]
wins = list(zip(ends[1:-1], ends[2:]))  # skip the first (warm-up) window
tot, cnt = defaultdict(float), defaultdict(int)
span = 0.0
for a, b in wins:
    span += (int(rows[b]["End_Timestamp"]) - int(rows[a]["End_Timestamp"])) / 1e6
    for r in rows[a + 1:b + 1]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        tot[r["Kernel_Name"]] += d
        cnt[r["Kernel_Name"]] += 1
n = len(wins)
busy = sum(tot.values()) / n
print(f"{n} steady-state steps: wall {span / n:.3f} ms/step, kernel-busy {busy:.3f} ms/step, "
      f"{sum(cnt.values()) / n:.0f} launches/step")
for k in sorted(tot, key=lambda k: -tot[k])[:top]:
    print(f"{tot[k] / n:8.3f} ms {100 * tot[k] / n / busy:5.1f}%  x{cnt[k] / n:4.1f}  avg {tot[k] / cnt[k] * 1e3:8.1f} us  {k[:110]}")
