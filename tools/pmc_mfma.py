"""MFMA utilisation of bench.py's probe kernel from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE (tools/gpu_pmc.sh style run):
    python tools/pmc_mfma.py gpurun_out/<tag>/pmc_mfma [kernel fragment]
Per launch of the matching kernel: busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs x 4 SIMDs x
GRBM_GUI_ACTIVE / 8) (GRBM_GUI_ACTIVE is summed over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back'; the
MFMA counter counts SIMD cycles, 32 per v_mfma_f32_32x32x16_bf16), and the effective clock."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
frag = sys.argv[2] if len(sys.argv) > 2 else "gemm_pipe_kernel<(anonymousnamespace)::PipeCfg<256,256,4,4,2,64,3,0,0>"
# the conv1 implicit GEMM's grid (threads) for the default probe; any grid for another kernel
GRID = ((32 * 4799 + 255) // 256) * ((512 + 255) // 256) * 1024 if len(sys.argv) <= 2 else 0
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace(" ", "")
        if frag not in name or (GRID and int(r.get("Grid_Size", 0) or 0) != GRID):
            continue
        vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = []
for d, c in vals.items():
    if {"SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"} <= set(c):
        cyc = c["GRBM_GUI_ACTIVE"] / 8.0
        rows.append(dict(mfma_busy_frac=c["SQ_VALU_MFMA_BUSY_CYCLES"] / (256 * 4 * cyc), gui_cycles=cyc,
                         sq_busy_cu_cycles=c.get("SQ_BUSY_CU_CYCLES")))
out = {"kernel_match": frag, "grid_threads": GRID, "launches": len(rows)}
if rows:
    out["mfma_busy_frac_avg"] = sum(r["mfma_busy_frac"] for r in rows) / len(rows)
    out["gui_active_cycles_avg"] = sum(r["gui_cycles"] for r in rows) / len(rows)
print(json.dumps(out, indent=1))
