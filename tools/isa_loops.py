"""Loops of one kernel in a hipcc -S listing: for every backward branch, the
instruction mix between its target label and the branch (memory ops, scratch,
SGPR-spill lane moves). Finds spill/scratch traffic inside hot gather loops.
usage: python tools/isa_loops.py listing.s kernel_substring"""
import re
import sys
from collections import Counter

path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end + 1]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\w+):", l)
    if m:
        labels[m.group(1)] = i
keys = ("buffer_load", "global_load", "global_store", "scratch_load", "scratch_store", "ds_read", "ds_write",
        "v_readlane", "v_writelane", "s_waitcnt", "v_")
for i, l in enumerate(body):
    m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)", l) or re.match(r"^\s+s_branch\s+(\.LBB\w+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        a = labels[m.group(1)]
        c = Counter()
        n = 0
        for x in body[a:i + 1]:
            x = x.strip()
            if not x or x.startswith(";") or x.startswith("."):
                continue
            n += 1
            op = x.split()[0]
            for k in keys:
                if op.startswith(k):
                    c[k] += 1
                    break
        if c["buffer_load"] or c["scratch_load"] or c["scratch_store"]:
            print(f"loop {m.group(1)} lines {a}-{i} insts {n}: " + " ".join(f"{k}={v}" for k, v in c.items()))
