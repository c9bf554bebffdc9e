#!/bin/bash
# the GPU suite up to 3 times; on a host crash, a backtrace from the core file (tools/core_rip.py)
mkdir -p gpurun_out/fl
ulimit -c unlimited
for i in 1 2 3 4 5 6 7 8; do
  rm -f core core.*
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fl/suite$i.log 2>&1
  rc=$?
  echo "suite $i rc=$rc"
  if [ $rc -ne 0 ]; then
    c=$(ls core core.* 2>/dev/null | head -1)
    if [ -n "$c" ]; then timeout -k 10 120 python3 tools/core_rip.py $c > gpurun_out/fl/core.txt 2>&1; rm -f core core.*; fi
    exit 1
  fi
done
