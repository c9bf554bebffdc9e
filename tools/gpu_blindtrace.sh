#!/bin/bash
# pdcch_blind duration per library build: tools/gpu_blindtrace.sh <A.so> <B.so> ...
set -e
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  OUT=gpurun_out/bt/$i
  mkdir -p $OUT
  MI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --workload ue_dl --steps 2 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1 || echo "(bench exit $?)"
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; grep -E "pdcch|ctrl_llr" $f | cut -d, -f1-5
  i=$((i+1))
done
