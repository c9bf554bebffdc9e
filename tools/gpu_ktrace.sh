#!/bin/bash
# per-dispatch kernel trace of the default bench (and --workload ue_dl): tools/gpu_ktrace.sh <tag>
set -e
TAG=${1:-cur}
export TMPDIR=/tmp
for w in pdsch ue_dl; do
  OUT=gpurun_out/kt_$TAG/$w
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o tr -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
  cp $(find $OUT -name "*kernel_trace.csv" | head -1) gpurun_out/kt_$TAG/${w}_kernel_trace.csv
done
echo rc=0
