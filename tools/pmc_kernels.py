#!/usr/bin/env python3
"""Per-kernel table of a tools/gpu/e2e_pmc.sh run: time (kernel trace), HBM bytes per launch (2 x FETCH_SIZE +
WRITE_SIZE, MI355X_MICROARCH.md's gfx950 rule), SQ shares of wave time, LDS conflicts.  python3 tools/pmc_kernels.py
gpurun_out/pmc_<tag> [min_us]
(averages are over every launch of a kernel name, no-op launches included: a kernel whose later launches early-exit
shows its real launch's bytes and time diluted by the call count)"""
import collections
import csv
import glob
import sys

D = sys.argv[1]
MIN_US = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0


def short(n):
    n = n.replace("mi355::", "").replace("void ", "")
    return n.split("(")[0][:52]


def load(sub):
    f = glob.glob(f"{D}/{sub}/**/*counter_collection.csv", recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    if f:
        for r in csv.DictReader(open(f[0])):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


tr = {}
f = glob.glob(f"{D}/trace/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    tr[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
fe, wr, sq, ld = load("fetch"), load("write"), load("sq"), load("lds")
avg = lambda d, c: sum(d[c]) / len(d[c]) if d.get(c) else float("nan")
print(f"{'kernel':52s} {'calls':>5s} {'avg us':>8s} {'rd MB':>8s} {'wr MB':>8s} {'TB/s':>6s} {'valu%':>6s} {'wait%':>6s} "
      f"{'lds/vmem':>8s} {'ldsconf%':>8s}")
for k, (calls, us) in sorted(tr.items(), key=lambda kv: -kv[1][0] * kv[1][1]):
    if us < MIN_US:
        continue
    rd = 2 * avg(fe[k], "FETCH_SIZE") / 1024
    w = avg(wr[k], "WRITE_SIZE") / 1024
    wc = avg(sq[k], "SQ_WAVE_CYCLES")
    wait = 100 * avg(sq[k], "SQ_WAIT_ANY") / wc if wc else float("nan")
    valu = 100 * avg(ld[k], "SQ_ACTIVE_INST_VALU") / wc if wc else float("nan")
    vm = avg(sq[k], "SQ_INSTS_VMEM_RD") + avg(sq[k], "SQ_INSTS_VMEM_WR")
    lds = avg(ld[k], "SQ_INSTS_LDS")
    act = avg(ld[k], "SQ_LDS_IDX_ACTIVE") if ld.get(k) else 0.0
    conf = 100 * avg(ld[k], "SQ_LDS_BANK_CONFLICT") / act if act else float("nan")
    print(f"{k:52s} {calls:5d} {us:8.1f} {rd:8.1f} {w:8.1f} {(rd + w) / us:6.2f} {valu:6.1f} {wait:6.1f} "
          f"{lds / vm if vm else float('nan'):8.2f} {conf:8.1f}")
