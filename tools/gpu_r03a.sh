#!/bin/bash
# r03a: state check at round start -- smoke, GPU suite, default bench
mkdir -p gpurun_out/r03a
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r03a/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a/gputest.log 2>&1 || { echo suite failed; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { echo bench failed; exit 1; }
echo rc=0
