#!/usr/bin/env python3
"""Per-basic-block instruction tally of one kernel in a hipcc -S listing.

usage: asm_blocks.py <file.s> <kernel-symbol-substring> [first_line last_line]
Prints each block (label, listing line) with its VALU / SALU / DS / VMEM / wait
counts, so the hot loop's per-tile instruction budget can be read off by hand.
"""
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l and l.rstrip().endswith(":")
                 or (l.startswith("_Z") and sym in l.split(":")[0]))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 30
    blocks, cur = [], None
    for i in range(start, end):
        l = lines[i]
        if re.match(r"^\.LBB\w+:|^; %bb\.\d+:", l):
            cur = {"name": l.split()[0].rstrip(":") if l.startswith(".") else l.split()[1].rstrip(":"),
                   "line": i - start + 1, "v": 0, "s": 0, "ds": 0, "vm": 0, "wait": 0, "br": ""}
            blocks.append(cur)
            continue
        t = l.strip()
        if cur is None or not t or t.startswith(";") or t.startswith("."):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            cur["v"] += 1
        elif op.startswith("s_waitcnt"):
            cur["wait"] += 1
        elif op.startswith("s_cbranch") or op.startswith("s_branch"):
            cur["br"] += op.replace("s_cbranch_", "").replace("s_branch", "jmp") + ">" + t.split()[-1] + " "
            cur["s"] += 1
        elif op.startswith("s_"):
            cur["s"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            cur["vm"] += 1
    tv = ts = 0
    for b in blocks:
        if not (lo <= b["line"] <= hi):
            continue
        tv += b["v"]
        ts += b["s"]
        print(f"{b['name']:<12} {b['line']:5d}  v={b['v']:3d} s={b['s']:3d} ds={b['ds']:2d} vm={b['vm']:2d} "
              f"w={b['wait']}  {b['br']}")
    print(f"total v={tv} s={ts}")


if __name__ == "__main__":
    main()
