#!/usr/bin/env python3
"""Per-kernel summary of tools/e2e_sq.sh counters (profiles/r02h_e2e/): time from SQ_BUSY_CYCLES (32 SEs, 2.4 GHz),
VALU-active / issue-wait / memory-wait shares of wave time, FETCH_SIZE and WRITE_SIZE per launch."""
import collections
import csv
import sys

D = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02h_e2e"


def load(name):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{D}/{name}_counters.csv")):
        k = r["Kernel_Name"].split("(")[0].replace("mi355::", "")[:44]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


sq, fe, wr = load("sq"), load("fetch"), load("write")
avg = lambda d, c: sum(d[c]) / len(d[c]) if d[c] else 0.0
print(f"{'kernel':44s} {'busy us':>8s} {'valu%':>6s} {'issue-wait%':>11s} {'mem-wait%':>9s} {'fetch MB':>9s} {'write MB':>9s}")
for k, v in sq.items():
    wc = avg(v, "SQ_WAVE_CYCLES")
    if wc < 1e6:
        continue
    print(f"{k:44s} {avg(v, 'SQ_BUSY_CYCLES') / 32 / 2.4e3:8.1f} {100 * avg(v, 'SQ_ACTIVE_INST_VALU') / wc:6.1f} "
          f"{100 * avg(v, 'SQ_WAIT_INST_ANY') / wc:11.1f} {100 * avg(v, 'SQ_WAIT_ANY') / wc:9.1f} "
          f"{avg(fe[k], 'FETCH_SIZE') / 1024:9.0f} {avg(wr[k], 'WRITE_SIZE') / 1024:9.0f}")
