"""Summarise rocprofv3 PMC passes for the dominant kernel (bg_kernel).

usage: python tools/pmc_traffic.py <pmc_root_dir> <workload> [--kernel bg_kernel] [--write profiles/pmc_<workload>.json]

Reads every *counter_collection.csv under <pmc_root_dir>, keeps dispatches whose
kernel name contains --kernel, averages each counter per dispatch, and derives
HBM bytes per launch per MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts half the bytes of a
streaming read (x2 correction); WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def collect(root, kernel):
    per = defaultdict(lambda: defaultdict(float))  # (file, dispatch) -> counter -> value
    grid = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row.get("Kernel_Name", ""):
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
                grid[key] = int(float(row.get("Grid_Size") or 0))
    # keep the main (largest-grid) launches only: a step also launches the same
    # kernel on the few flush columns
    gmax = max(grid.values()) if grid else 0
    per = {k: v for k, v in per.items() if grid.get(k, 0) == gmax}
    sums, counts = defaultdict(float), defaultdict(int)
    for vals in per.values():
        for k, v in vals.items():
            sums[k] += v
            counts[k] += 1
    return {k: sums[k] / counts[k] for k in sums}, len(per)


def main():
    root, workload = sys.argv[1], sys.argv[2]
    kernel = "bg_kernel"
    out = None
    a = sys.argv[3:]
    for i, t in enumerate(a):
        if t == "--kernel":
            kernel = a[i + 1]
        if t == "--write":
            out = a[i + 1]
    avg, n = collect(root, kernel)
    res = {"workload": workload, "kernel": kernel, "dispatch_samples": n, "counters_avg_per_dispatch": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        rd = avg["FETCH_SIZE"] * 1024 * 2     # gfx950 FETCH_SIZE half-count correction
        wr = avg["WRITE_SIZE"] * 1024
        res.update(hbm_read_bytes_per_launch=rd, hbm_write_bytes_per_launch=wr, hbm_bytes_per_launch=rd + wr,
                   correction="FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg:
        res["mfma_busy_frac"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (avg["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
    if "SQ_WAVE_CYCLES" in avg:
        w = avg["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in avg:
                res[k + "_frac"] = avg[k] / w
    txt = json.dumps(res, indent=1, sort_keys=True)
    print(txt)
    if out:
        with open(out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
