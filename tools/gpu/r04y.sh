#!/bin/bash
# r04y: round-4 closing check: GPU suite, smoke, default bench (roofline + CPU baseline), ue_dl / tdec / siso_qpsk
# benches, drop-in latency, e2e kernel statistics
set -e
OUT=gpurun_out/r04y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/suite.log 2>&1 || { rc=$?; echo suite rc=$rc; tail -30 $OUT/suite.log; exit $rc; }
tail -1 $OUT/suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 900 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python3 -u bench.py --workload ue_dl --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/pdsch_same_box.json 2> $OUT/pdsch_same_box.err
timeout -k 10 300 python3 -u bench.py --workload tdec --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/tdec.json 2> $OUT/tdec.err
timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 1000 > $OUT/dropin_lat.json 2> $OUT/dropin_lat.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_tr.json 2> $OUT/e2e_tr.err
echo rc=0
