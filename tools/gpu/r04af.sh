#!/bin/bash
# r04af: one-launch softbuffer resets, event-ordered drop-in resets: GPU suite, smoke, drop-in latency
set -e
OUT=gpurun_out/r04af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/suite.log 2>&1 || { rc=$?; echo suite rc=$rc; tail -30 $OUT/suite.log; exit $rc; }
tail -1 $OUT/suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 300 python3 -u tools/dropin_lat.py 1000 > $OUT/dropin_lat.json 2> $OUT/dropin_lat.err
echo rc=0
