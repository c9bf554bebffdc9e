#!/usr/bin/env python3
"""Summarise a tools/gpu_r03d.sh-style run (rocprofv3 CSVs under gpurun_out/<tag>/) into profiles/<tag>_pmc.json:

* calibration: FETCH_SIZE / WRITE_SIZE per launch of tools/microbench/fetch_calib against the bytes each pattern
  moves (1 GiB buffer, Infinity Cache evicted before every launch) -> one correction factor per access pattern;
* e2e: per kernel of the default bench step (2,048 TM4 subframes) the average launch time (kernel trace), FETCH_SIZE
  and WRITE_SIZE per launch and the corrected HBM bytes (reads x the coalesced-pattern factor, writes x 1);
* lds: SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT (extra cycles), SQ_LDS_IDX_ACTIVE (all LDS-array cycles) and
  SQ_WAIT_INST_LDS per launch of the find_and_decode workload's kernels.

usage: tools/r03_pmc_summary.py <tag>   (reads gpurun_out/<tag>, writes profiles/<tag>_pmc.json)"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    n = name.replace("void ", "")
    n = n.split("(")[0] if not n.startswith("mi355::(anonymous") else n.split(")::", 1)[-1].split("(")[0]
    return n.strip()


def per_kernel(path: str, counters=None):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    seen = set()
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if counters and r["Counter_Name"] not in counters:
            continue
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (k, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            calls[k] += 1
    return d, calls


def main(tag: str):
    base = os.path.join(ROOT, "gpurun_out", tag)
    out = {"tag": tag, "units": "bytes per launch (FETCH_SIZE / WRITE_SIZE are KiB in rocprofv3 7.2; x 1024)"}
    # ---- calibration
    moved = {}
    for line in open(os.path.join(base, "cal_fetch.log")):
        p = line.split()
        if len(p) >= 3 and p[1] == "bytes":
            moved[p[0]] = int(p[2])
    cal = {}
    for f, cn in (("cal_fetch/cal_fetch_counter_collection.csv", "FETCH_SIZE"),
                  ("cal_write/cal_write_counter_collection.csv", "WRITE_SIZE")):
        for r in csv.DictReader(open(os.path.join(base, f))):
            k = short(r["Kernel_Name"])
            name = {"rd_stream<unsigned int>": "rd_b32", "rd_stream<HIP_vector_type<unsigned int, 2u> >": "rd_b64",
                    "rd_stream<HIP_vector_type<unsigned int, 4u> >": "rd_b128",
                    "wr_stream<unsigned int>": "wr_b32", "wr_stream<HIP_vector_type<unsigned int, 2u> >": "wr_b64",
                    "wr_stream<HIP_vector_type<unsigned int, 4u> >": "wr_b128",
                    "wr_stream<unsigned short>": "wr_b16"}.get(k, k)
            if name not in moved or (cn == "FETCH_SIZE") != name.startswith("rd"):
                continue
            cal[name] = {"bytes": moved[name], cn: float(r["Counter_Value"]) * 1024,
                         "counted_over_moved": round(float(r["Counter_Value"]) * 1024 / moved[name], 4)}
    out["calibration"] = {"patterns": cal, "rule": "coalesced reads of 4, 8 or 16 B per lane (whole or half rows): "
                          "FETCH_SIZE counts 1/2 of the bytes -> x 2; random 8-B gathers: one 64-B line counted per "
                          "gather (x 1 = real line traffic); WRITE_SIZE exact for 2-16 B per lane stores"}
    # ---- e2e per kernel
    fe, fcalls = per_kernel(os.path.join(base, "e2e_fetch/fetch_counter_collection.csv"), {"FETCH_SIZE"})
    wr, wcalls = per_kernel(os.path.join(base, "e2e_write/write_counter_collection.csv"), {"WRITE_SIZE"})
    st = {}
    for r in csv.DictReader(open(os.path.join(base, "e2e_trace/trace_kernel_stats.csv"))):
        st[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
    e2e = {}
    for k in fe:
        f = fe[k]["FETCH_SIZE"] * 1024 / max(1, fcalls[k])
        w = wr[k]["WRITE_SIZE"] * 1024 / max(1, wcalls[k]) if k in wr else 0.0
        if f + w < 1e6:
            continue
        e = {"fetch_size_bytes": round(f), "write_size_bytes": round(w), "hbm_bytes_corrected": round(2 * f + w)}
        if k in st:
            e.update(st[k])
            e["achieved_TBps_corrected"] = round((2 * f + w) / (st[k]["avg_us"] * 1e-6) / 1e12, 2)
        e2e[k] = e
    out["e2e_step"] = dict(sorted(e2e.items(), key=lambda kv: -kv[1]["hbm_bytes_corrected"]))
    # ---- LDS
    ld, lcalls = per_kernel(os.path.join(base, "lds/lds_counter_collection.csv"))
    lds = {}
    for k, v in ld.items():
        if not v.get("SQ_INSTS_LDS"):
            continue
        c = max(1, lcalls[k])
        lds[k] = {"launches": c, "waves": round(v["SQ_WAVES"] / c), "lds_instr": round(v["SQ_INSTS_LDS"] / c),
                  "bank_conflict_cycles": round(v["SQ_LDS_BANK_CONFLICT"] / c),
                  "lds_active_cycles": round(v["SQ_LDS_IDX_ACTIVE"] / c),
                  "conflict_share": round(v["SQ_LDS_BANK_CONFLICT"] / max(1.0, v["SQ_LDS_IDX_ACTIVE"]), 4),
                  "wait_inst_lds": round(v["SQ_WAIT_INST_LDS"] / c), "busy_cycles": round(v["SQ_BUSY_CYCLES"] / c)}
    out["lds_find_and_decode"] = dict(sorted(lds.items(), key=lambda kv: -kv[1]["bank_conflict_cycles"]))
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(path)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r03d")
