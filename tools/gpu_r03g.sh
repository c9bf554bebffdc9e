#!/bin/bash
# r03g: round-3 closing check on the restored head: full GPU suite, smoke, benches (default with CPU baseline,
# ue_dl, tdec, siso_qpsk) and rocprofv3 kernel statistics of the pdsch and ue_dl benches
set -e
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_suite.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -k 10 300 python -u bench.py --workload tdec > $OUT/tdec.json 2> $OUT/tdec.err
timeout -k 10 300 python -u bench.py --workload siso_qpsk > $OUT/siso.json 2> $OUT/siso.err
bash tools/gpu_stats.sh r03g > /dev/null
echo rc=0
