#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over the MAP kernel's probe launches (tools/map_pmc.py) for each mode, plus a kernel
# trace (run under gpurun): tools/gpu/map_pmc.sh <tag> [modes...]  -> gpurun_out/<tag>/<mode>/{fetch,write,trace}
# then locally: python3 tools/map_pmc_summary.py gpurun_out/<tag>/<mode> <mode> <tag>
set -e
TAG=$1; shift
MODES=${*:-e2e siso tdec}
export TMPDIR=/tmp
for m in $MODES; do
  OUT=gpurun_out/$TAG/$m
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k -- python3 tools/map_pmc.py $m > $OUT/trace.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex tdec_win_halfit --output-format csv -d $OUT/fetch -o f -- python3 tools/map_pmc.py $m > $OUT/fetch.log 2>&1
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex tdec_win_halfit --output-format csv -d $OUT/write -o w -- python3 tools/map_pmc.py $m > $OUT/write.log 2>&1
  tail -1 $OUT/write.log
done
echo rc=0
