#!/bin/bash
# r02j: GPU suite (host-crash backtrace on failure), default bench, e2e kernel stats
mkdir -p gpurun_out/r02j
ulimit -c unlimited
rm -f core core.*
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02j/gputest.log 2>&1
rc=$?
if [ $rc -ne 0 ]; then
  c=$(ls core core.* 2>/dev/null | head -1)
  if [ -n "$c" ]; then timeout -k 10 120 python3 tools/core_rip.py $c > gpurun_out/r02j/core.txt 2>&1; rm -f core core.*; fi
  echo "suite rc=$rc"; exit 1
fi
timeout -k 10 300 python -u bench.py > gpurun_out/r02j/bench.json 2> gpurun_out/r02j/bench.err && bash tools/e2e_stats.sh r02j
echo rc=$?
