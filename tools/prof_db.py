"""Summarise a rocprofv3 --kernel-trace SQLite output (run_results.db): per-kernel stats (the
columns of rocprofv3 --stats' kernel_stats.csv) and per-(kernel, grid, workgroup) launch
statistics (a bench step launches one kernel symbol with several grids: the stream body, the
flush tail, per-workload geometries).

usage: python tools/prof_db.py <run_results.db> [--stats out_kernel_stats.csv] [--grid out_by_grid.txt]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def load(path):
    con = sqlite3.connect(path)
    return con.execute("select name, grid_x, workgroup_x, duration, lds_size, vgpr_count, sgpr_count, start "
                       "from kernels order by start").fetchall()


def stats(rows):
    d = defaultdict(list)
    for name, *_r in rows:
        d[name].append(_r[2])
    tot = sum(sum(v) for v in d.values()) or 1
    out = []
    for name, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        n = len(v)
        mean = sum(v) / n
        sd = (sum((x - mean) ** 2 for x in v) / n) ** 0.5
        out.append([name, n, sum(v), round(mean, 3), round(100.0 * sum(v) / tot, 4), min(v), max(v), round(sd, 3)])
    return out


def by_grid(rows):
    d = defaultdict(list)
    meta = {}
    for name, gx, wx, dur, lds, vg, sg, _ in rows:
        d[(name, gx, wx)].append(dur)
        meta[(name, gx, wx)] = (lds, vg, sg)
    lines = []
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        n = len(v)
        lds, vg, sg = meta[k]
        lines.append(f"{k[0][:70]:70s} grid {k[1]:>9d} wg {k[2]:>5d} calls {n:>6d} avg_us {sum(v) / n / 1e3:10.3f} "
                     f"min_us {min(v) / 1e3:9.3f} max_us {max(v) / 1e3:9.3f} total_ms {sum(v) / 1e6:9.3f} "
                     f"lds {lds} vgpr {vg} sgpr {sg}")
    return lines


if __name__ == "__main__":
    rows = load(sys.argv[1])
    args = sys.argv[2:]
    st = stats(rows)
    g = by_grid(rows)
    if "--stats" in args:
        with open(args[args.index("--stats") + 1], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
            w.writerows(st)
    if "--grid" in args:
        with open(args[args.index("--grid") + 1], "w") as f:
            f.write("\n".join(g) + "\n")
    for line in g[:40]:
        print(line)
