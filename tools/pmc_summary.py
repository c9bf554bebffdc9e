#!/usr/bin/env python3
"""Summarise a tools/profile_tdec.sh run into profiles/<tag>_* and profiles/r02_tdec_pmc.json (read by bench.py).

HBM bytes per MAP launch, as MI355X_MICROARCH.md's HBM section prescribes for gfx950: 2 x FETCH_SIZE (it counts
half the bytes of wide coalesced reads) + WRITE_SIZE (exact), both KB, each from its own --pmc pass.  The file is
keyed by the SHA-1 of the MAP kernel's sources (bench.map_kernel_hash): bench.py refuses a summary recorded on
other sources."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

TAG = sys.argv[1] if len(sys.argv) > 1 else "r02"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
P = os.path.join(ROOT, "gpurun_out", f"prof_{TAG}")
OUTD = os.path.join(ROOT, "profiles")
MAP = "tdec_win_halfit"
NCB, K = 65536, 6144


def counters(sub):
    f = glob.glob(os.path.join(P, sub, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        agg[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def per_kernel(agg, counter, pat=MAP):
    vals = [v for (k, c), vs in agg.items() if pat in k and c == counter for v in vs]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    import bench
    os.makedirs(OUTD, exist_ok=True)
    for sub, name in (("trace", "kernel_stats"), ("e2e", "e2e_kernel_stats")):
        f = glob.glob(os.path.join(P, sub, "**", "*kernel_stats.csv"), recursive=True)
        if f:
            shutil.copy(f[0], os.path.join(OUTD, f"{TAG}_{name}.csv"))
    fetch, nf = per_kernel(counters("fetch"), "FETCH_SIZE")
    write, nw = per_kernel(counters("write"), "WRITE_SIZE")
    sq = counters("sq")
    valu, _ = per_kernel(sq, "SQ_INSTS_VALU")
    waves, _ = per_kernel(sq, "SQ_WAVES")
    hbm = 2 * fetch * 1024 + write * 1024 if (fetch is not None and write is not None) else None
    res = {
        "tag": TAG, "kernel": MAP, "kernel_src_sha1": bench.map_kernel_hash(), "launch_ncb": NCB, "K": K,
        "fetch_size_kb_per_launch": fetch, "write_size_kb_per_launch": write, "launches_counted": [nf, nw],
        "hbm_bytes_per_launch": hbm,
        "hbm_rule": "2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md, HBM [CDNA4])",
        "valu_insts_per_launch": valu, "waves_per_launch": waves,
        "valu_lane_instr_per_cb_halfit": valu * 64 / NCB if valu else None,
    }
    json.dump(res, open(os.path.join(OUTD, "r02_tdec_pmc.json"), "w"), indent=1)
    json.dump(res, open(os.path.join(OUTD, f"{TAG}_pmc_summary.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
