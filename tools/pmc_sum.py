"""Per-kernel averages of PMC counters from tools/pmc_one.sh output dirs (one line per tag)."""
import collections, csv, glob, json, sys

def summarize(d, kernel="hx_kernel"):
    agg = {}
    for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv")):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        by = collections.defaultdict(list)
        for (di, c), v in per.items():
            by[c].append(v)
        for c, v in by.items():
            agg[c] = sum(v[1:]) / (len(v) - 1) if len(v) > 1 else v[0]
    return agg

if __name__ == "__main__":
    args = sys.argv[1:]
    kernel = "hx_kernel"
    if args and args[0] == "--kernel":
        kernel, args = args[1], args[2:]
    for d in args:
        a = summarize(d, kernel)
        w = a.get("SQ_WAVE_CYCLES", 1)
        print(d, json.dumps({k: float(f"{v:.4g}") for k, v in sorted(a.items())}))
        if "SQ_WAIT_ANY" in a:
            print("   wait_any %.2f wait_inst %.2f active %.2f  mfma_busy/gui %.3f" % (
                a["SQ_WAIT_ANY"] / w, a.get("SQ_WAIT_INST_ANY", 0) / w, a.get("SQ_ACTIVE_INST_ANY", 0) / w,
                a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, a.get("GRBM_GUI_ACTIVE", 1)) / 1024 * 8))
