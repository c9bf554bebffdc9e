#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S listing:  tools/isa_mix.py <file.s> <symbol substring> [--loops]

Prints the static instruction counts by opcode, the register / LDS / occupancy metadata, and with --loops the
mix inside each basic block that ends in a backward branch (the unrolled segment loops)."""
import re
import sys
from collections import Counter


def blocks(body):
    cur, name = [], "entry"
    for l in body:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            yield name, cur
            cur, name = [], s[:-1]
            continue
        cur.append(s)
    yield name, cur


def ops(lines):
    c = Counter()
    for s in lines:
        t = s.split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        c[t[0]] += 1
    return c


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [k for k, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l.split(":")[0]]
    if not starts:
        sys.exit("no symbol matching " + sym)
    i = starts[0]
    print(lines[i].split(":")[0])
    j = i
    while not lines[j].strip().startswith(".Lfunc_end"):
        j += 1
    body = lines[i:j]
    c = ops(body)
    print("total", sum(c.values()))
    for k, v in c.most_common(40):
        print(f"  {k:32s} {v}")
    for l in lines[j : j + 60]:
        if re.search(r"NumVgprs|NumAgprs|ScratchSize|Occupancy|LDSByteSize|NumSgprs|SpillCount", l):
            print(l.strip())
    if "--loops" in sys.argv:
        for name, bl in blocks(body):
            br = [s for s in bl if s.startswith("s_cbranch") or s.startswith("s_branch")]
            c = ops(bl)
            n = sum(c.values())
            if n < 200:
                continue
            valu = sum(v for k, v in c.items() if k.startswith("v_") and not k.startswith("v_readfirstlane"))
            vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
            wait = sum(v for k, v in c.items() if k.startswith("s_waitcnt"))
            print(f"block {name}: {n} instr, VALU {valu}, VMEM {vmem}, waitcnt {wait}, ends {br[-1] if br else '-'}")
            for k, v in c.most_common(14):
                print(f"    {k:30s} {v}")


if __name__ == "__main__":
    main()
