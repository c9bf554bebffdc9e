#!/bin/bash
# dlsch_rm_rx duration per library build (e2e bench, rocprofv3 stats): tools/gpu_rmtrace.sh <A.so> <B.so> ...
set -e
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  OUT=gpurun_out/rt/$i
  mkdir -p $OUT
  MI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $lib $(grep -o '"ms_per_step": [0-9.]*' $OUT/log)"; grep -E "dlsch_rm_rx|tdec_win_halfit<16, 8, 0" $f | cut -d, -f1-5
  i=$((i+1))
done
