"""Per-(kernel, grid) launch statistics from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_summary.py <run_kernel_trace.csv> [--write out.json]

rocprofv3 --stats averages every launch of one kernel symbol together; a bench
step launches bg_kernel twice (the stream body on the full grid and the short
flush tail), so the dominant launch's duration is read per grid size here.
"""
import csv
import json
import sys
from collections import defaultdict


def summarize(path):
    d = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
            d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (name, grid, wg), v in d.items():
        rows.append({"kernel": name, "grid_x": grid, "workgroup_x": wg, "calls": len(v),
                     "avg_ns": sum(v) / len(v), "min_ns": min(v), "max_ns": max(v), "total_ns": sum(v)})
    rows.sort(key=lambda r: -r["total_ns"])
    return rows


def main():
    rows = summarize(sys.argv[1])
    for r in rows:
        print(f'{r["total_ns"] / 1e6:10.3f} ms {r["calls"]:5d} x {r["avg_ns"] / 1e3:10.2f} us  grid {r["grid_x"]:8d}'
              f'  wg {r["workgroup_x"]:5d}  {r["kernel"][:90]}')
    if "--write" in sys.argv:
        with open(sys.argv[sys.argv.index("--write") + 1], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
