"""Step timeline of a bench run from a rocprofv3 --kernel-trace CSV: for every launch of the dominant
streaming kernel (KEY, default hxt_kernel), the kernels that follow it up to the next one, with their
durations and the idle gaps between consecutive dispatches (ns).  Summarises the median step.

usage: python tools/trace_steps.py <kernel_trace.csv> [KEY]
"""
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "hxt_kernel"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
    rows.sort()
    idx = [i for i, r in enumerate(rows) if key in r[2]]
    steps = []
    for a, b in zip(idx, idx[1:]):
        seq = rows[a:b + 1]
        step_ns = seq[-1][0] - seq[0][0]
        parts = []
        for (s0, e0, n0), (s1, e1, n1) in zip(seq, seq[1:]):
            parts.append((n0, e0 - s0, s1 - e0))
        steps.append((step_ns, parts))
    if not steps:
        print("no steps")
        return
    med = statistics.median(s for s, _ in steps)
    print(f"{len(steps)} steps of '{key}': start-to-start median {med / 1e3:.2f} us, min {min(s for s, _ in steps) / 1e3:.2f}")
    best = min(steps, key=lambda s: abs(s[0] - med))
    for name, dur, gap in best[1]:
        print(f"  {dur / 1e3:9.2f} us  then gap {gap / 1e3:7.2f} us  {name}")


if __name__ == "__main__":
    main()
