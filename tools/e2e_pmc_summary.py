#!/usr/bin/env python3
"""Summarise tools/profile_e2e.sh: per kernel of the TM4 ue_dl chain, average duration (trace), HBM-side
bytes (FETCH_SIZE + WRITE_SIZE, raw -- FETCH_SIZE under-reports wide coalesced reads by 2x on gfx950, see
MI355X_MICROARCH.md), VALU instructions, wave-cycle split and L2 hit rate.  Writes profiles/<tag>_e2e_pmc.json."""
import collections
import csv
import glob
import json
import os
import sys

TAG = sys.argv[1] if len(sys.argv) > 1 else "cur"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "gpurun_out", f"pmc_{TAG}")


def short(name):
    n = name.replace("mi355::", "").replace("void ", "")
    return n.split("(")[0]


def counters(sub):
    f = glob.glob(os.path.join(P, sub, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(list)
    if not f:
        return agg
    for r in csv.DictReader(open(f[0])):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main():
    stats = glob.glob(os.path.join(P, "trace", "**", "*kernel_stats.csv"), recursive=True)
    dur = {}
    for r in csv.DictReader(open(stats[0])):
        dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    allc = {}
    for sub in ("fetch", "write", "sq", "tcc"):
        allc.update(counters(sub))
    out = {}
    for k, (calls, us) in sorted(dur.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
        def avg(c):
            v = allc.get((k, c))
            return sum(v) / len(v) if v else None
        fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
        row = {"calls": calls, "avg_us": round(us, 1)}
        if fetch is not None and write is not None:
            row["fetch_MB"] = round(fetch / 1024, 2)
            row["write_MB"] = round(write / 1024, 2)
            row["raw_GBps"] = round((fetch + write) * 1024 / (us * 1e3), 1)
        for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            v = avg(c)
            if v is not None:
                row[c] = v
        wc, wa, wi, ac = (avg(c) for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
        if wc:
            row["wait_frac"] = round(wa / wc, 3)
            row["issue_stall_frac"] = round(wi / wc, 3)
            row["active_frac"] = round(ac / wc, 3)
        h, m = avg("TCC_HIT_sum"), avg("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            row["l2_hit"] = round(h / (h + m), 3)
        out[k] = row
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", f"{TAG}_e2e_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    for k, r in out.items():
        print(f"{k[:40]:40s} {json.dumps(r)}")


if __name__ == "__main__":
    main()
