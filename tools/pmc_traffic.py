"""Per-launch HBM traffic of bench.py's probe kernel from rocprofv3 --pmc passes (tools/gpu_pmc.sh):
    python tools/pmc_traffic.py gpurun_out/<tag>/pmc > profiles/pmc_traffic.json
FETCH_SIZE (KB) is doubled (gfx950: it reports half of a 16-B/lane streaming read, MI355X_MICROARCH.md
'HBM'), WRITE_SIZE (KB) is exact; traffic = 1024 * (2 * FETCH + WRITE) bytes, averaged over the probe's
launches (matched by kernel-name fragment and grid size)."""
import csv
import glob
import json
import sys

root = sys.argv[1]
MATCH = "gemm_pipe_kernel<(anonymousnamespace)::PipeCfg<256,256,4,4,2,64,3,1,1>"  # (the conv1 variant of the train step, v23)
SHAPE = (32 * 4799, 512, 1536)
GRID = ((SHAPE[0] + 255) // 256) * ((SHAPE[1] + 255) // 256) * 1024  # blocks x threads


def counter(name):
    vals = []
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == name and MATCH in r["Kernel_Name"].replace(" ", "") and int(r["Grid_Size"]) == GRID:
                vals.append(float(r["Counter_Value"]))
    return vals


fetch, write = counter("FETCH_SIZE"), counter("WRITE_SIZE")
if not fetch or not write:
    sys.exit(f"no probe launches found (fetch {len(fetch)}, write {len(write)})")
f_kb, w_kb = sum(fetch) / len(fetch), sum(write) / len(write)
out = {"kernel_match": "gemm_pipe_kernel<PipeCfg<256,256,4,4,2,64,3,1,1>,bf16>", "shape": list(SHAPE),
       "fetch_kb_raw": f_kb, "write_kb": w_kb, "launches": [len(fetch), len(write)],
       "traffic_bytes_per_launch": int(1024 * (2 * f_kb + w_kb)),
       "algorithmic_bytes_per_launch": 2 * (32 * 9599 * 512 + 512 * 1536 + SHAPE[0] * 512)}
print(json.dumps(out, indent=1))
