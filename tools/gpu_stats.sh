#!/bin/bash
# rocprofv3 kernel statistics of the default bench and of --workload ue_dl (current build): tools/gpu_stats.sh <tag>
set -e
TAG=${1:-cur}
export TMPDIR=/tmp
for w in pdsch ue_dl; do
  OUT=gpurun_out/st_$TAG/$w
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
  cp $(find $OUT -name "*kernel_stats.csv" | head -1) gpurun_out/st_$TAG/${w}_kernel_stats.csv
done
echo rc=0
