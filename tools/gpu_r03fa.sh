#!/bin/bash
# r03f (part A): round-3 final check -- full GPU suite, smoke, MAP kernel PMC re-keyed to the current sources
set -e
OUT=gpurun_out/r03f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_suite.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $OUT/smoke.log 2>&1
bash tools/profile_tdec.sh r03f > $OUT/profile_tdec.log 2>&1
echo rc=0
