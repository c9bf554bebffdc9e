#!/usr/bin/env python3
"""Kernel timeline (with GPU idle gaps) of the last find_and_decode step of a tools/trace_uedl.sh run: from the first
kernel after the previous step's last DL-SCH epilogue to the step's own last epilogue (each step ends with one
epilogue per chunk: --chunks, default 2).  -v prints every kernel, otherwise only gaps > 20 us and kernels > 100 us."""
import csv
import glob
import sys

tag = next((a for a in sys.argv[1:] if not a.startswith("-")), "cur")
nch = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--chunks=")), 2)
f = glob.glob(f"gpurun_out/tu_{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
eps = [i for i, r in enumerate(rows) if "dlsch_tb_epilogue" in r["Kernel_Name"]]
last = eps[-1]
first = eps[-1 - nch] + 1 if len(eps) > nch else 0
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
