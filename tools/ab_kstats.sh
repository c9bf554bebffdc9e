#!/bin/bash
# Per-kernel A/B of two in-tree library builds on one box (run under gpurun):
#   tools/ab_kstats.sh <A.so> <B.so> <kernel-substring>...  -> average duration of each named kernel, A B A B
set -e
A=$1; B=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/abk
n=0
for lib in $A $B $A $B; do
  n=$((n+1))
  MI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abk/$n -o k -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > gpurun_out/abk/$n.log 2>&1
  python3 - "$lib" "gpurun_out/abk/$n" "$@" <<'PY'
import csv, glob, sys
lib, d, names = sys.argv[1], sys.argv[2], sys.argv[3:]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
out = []
for nm in names:
    v = [float(r["AverageNs"]) / 1e3 for r in rows if nm in r["Name"]]
    out.append(f"{nm} {max(v) if v else float('nan'):.1f}us")
print(lib, " ".join(out))
PY
done
