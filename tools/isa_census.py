#!/usr/bin/env python3
"""ISA census of one kernel in a hipcc -S listing: basic blocks, loops (backward branches), and per-loop
instruction counts by class (VALU / SALU / MFMA / LDS / VMEM / readlane+writelane / waitcnt).
usage: isa_census.py file.s kernel_substring"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op in ("v_readlane_b32", "v_writelane_b32", "v_readfirstlane_b32"):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "scratch" if op.startswith("scratch_") else "vmem"
    return "other"


def main(path, key):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", l) or (key in l and l.endswith(":") and l.startswith("_Z")))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    order = [cur]
    for l in lines[start + 1:end]:
        s = l.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        blocks[cur].append(s.split()[0])
    idx = {b: i for i, b in enumerate(order)}
    loops = []
    for b in order:
        for op_line in blocks[b]:
            pass
    # backward branches: a branch in block i to block j <= i
    for i, b in enumerate(order):
        pass
    raw = lines[start + 1:end]
    cur = "entry"
    for l in raw:
        s = l.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            continue
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", s)
        if m and m.group(2) in idx and idx[m.group(2)] <= idx[cur]:
            loops.append((m.group(2), cur))
    tot = Counter(classify(o) for b in order for o in blocks[b])
    print(f"kernel total: {sum(tot.values())} instrs", dict(tot))
    for head, tail in loops:
        body = order[idx[head]:idx[tail] + 1]
        c = Counter(classify(o) for b in body for o in blocks[b])
        n = sum(c.values())
        if n < 40:
            continue
        print(f"loop {head}..{tail} ({len(body)} blocks, {n} instrs):", dict(c))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
