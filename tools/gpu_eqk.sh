#!/bin/bash
# per-kernel average durations of the e2e bench for several builds: tools/gpu_eqk.sh <A.so> <B.so> ...
# (KF: comma-separated kernel-name fragments to print, default the equaliser / rate-dematching kernels)
set -e
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  OUT=gpurun_out/ek/$i
  mkdir -p $OUT
  MI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
  KF=${KF:-pdsch_eq_rm,dlsch_rm_rx,pdsch_eq_llr,csimax} python3 - $OUT $lib <<'PY'
import csv, glob, os, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
ms = re.search(r'"ms_per_step": ([0-9.]+)', open(sys.argv[1] + "/log").read())
print("==", sys.argv[2], ms.group(1) if ms else "?")
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in os.environ["KF"].split(",")):
        print("  ", r["Name"][:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
  i=$((i+1))
done
