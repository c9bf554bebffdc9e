#!/usr/bin/env python3
"""Kernel timeline (with GPU idle gaps) of the last find_and_decode step of a tools/trace_uedl.sh run."""
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
f = glob.glob(f"gpurun_out/tu_{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = max(i for i, r in enumerate(rows) if "dlsch_tb_epilogue" in r["Kernel_Name"])
first = max(i for i, r in enumerate(rows[:last]) if "ofdm_rx" in r["Kernel_Name"])
t0 = int(rows[first]["Start_Timestamp"])
prev_end, busy = t0, 0
agg = {}
for r in rows[first: last + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3
    name = r["Kernel_Name"].replace("mi355::", "").split("(")[0][:48]
    if "-v" in sys.argv or gap > 20 or (e - s) > 100e3:
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {name}")
    agg[name] = agg.get(name, 0) + (e - s) / 1e3
    busy += max(0, e - max(s, prev_end))
    prev_end = max(prev_end, e)
print(f"step span {(prev_end - t0) / 1e3:.1f} us, GPU busy {busy / 1e3:.1f} us")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:16]:
    print(f"  {k:50s} {v:9.1f} us")
