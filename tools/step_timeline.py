#!/usr/bin/env python3
"""Print the kernel timeline of the last decode step of a tools/trace_step.sh run (gaps included)."""
import csv
import glob
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
f = glob.glob(f"gpurun_out/tr_{tag}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# last fused mi355_ue_dl_decode_batch step: an ofdm_rx whose chest_estimate is followed by chest_noise (the
# bench's separate per-stage timing calls run without it)
fused = [i for i, r in enumerate(rows) if "ofdm_rx" in r["Kernel_Name"] and i + 2 < len(rows) and
         "chest_noise" in rows[i + 2]["Kernel_Name"]]
first = fused[-1]
last = [i for i, r in enumerate(rows) if "dlsch_tb_epilogue" in r["Kernel_Name"] and i > first][0]
t0 = int(rows[max(first - 1, 0)]["Start_Timestamp"])
prev_end = t0
for r in rows[max(first - 1, 0): last + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev_end) / 1e3
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:7.1f}  {r['Kernel_Name'].replace('mi355::', '')[:60]}")
    prev_end = max(prev_end, e)
print(f"step span {(prev_end - t0) / 1e3:.1f} us")
