"""Summarise a tools/gpu_ab_kernel.sh ab.txt: per (workload, variant) the kernel ms of every round and
the mean.  usage: python tools/ab_summary.py gpurun_out/<TAG>/ab.txt"""
import collections
import json
import sys

d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    w, j = line.split(" ", 1)
    j = json.loads(j)
    cfg = j["cfg"]
    name = cfg.get("GAR_LIB_PATH", "").split("/")[-1] or ",".join(f"{k}={v}" for k, v in cfg.items()) or "base"
    if "ms" in j:
        d[(w, name)].append(j["ms"])
for (w, name), v in sorted(d.items()):
    print(f"{w:6s} {name:28s} mean {sum(v) / len(v):.4f}  [" + " ".join(f"{x:.4f}" for x in v) + "]")
