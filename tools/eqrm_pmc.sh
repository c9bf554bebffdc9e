#!/bin/bash
# SQ counters (VALU / LDS / waves) of the e2e PDSCH kernels: pdsch_eq_rm vs pdsch_eq_llr + dlsch_rm_rx (run under gpurun)
set -e
OUT=gpurun_out/erpmc
mkdir -p $OUT
export TMPDIR=/tmp
for v in on off; do
  if [ $v = off ]; then export MI355_NO_EQRM=1; else unset MI355_NO_EQRM; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/$v -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log_$v 2>&1
done
unset MI355_NO_EQRM
python3 - <<'PY'
import csv, glob, collections
for v in ("on", "off"):
    f = glob.glob(f"gpurun_out/erpmc/{v}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if not any(k in n for k in ("pdsch_eq_rm", "dlsch_rm_rx", "pdsch_eq_llr")): continue
        n = n.split("(")[0][-24:]
        agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(n, r["Counter_Name"])] += 1
    for n, d in agg.items():
        k = max(c for (nn, _), c in cnt.items() if nn == n)
        print(v, n, {c: round(x / max(1, cnt[(n, c)] / (cnt[(n, c)] // max(1, k) or 1)), 0) for c, x in d.items()})
PY
