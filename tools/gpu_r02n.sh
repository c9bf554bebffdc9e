#!/bin/bash
# r02n round-end check: smoke, GPU suite, default bench, tdec (config 2) and ue_dl workloads
mkdir -p gpurun_out/r02n
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r02n/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r02n/gputest.log 2>&1 || { echo suite failed; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r02n/bench.json 2> gpurun_out/r02n/bench.err || { echo bench failed; exit 1; }
timeout -k 10 300 python -u bench.py --workload tdec > gpurun_out/r02n/tdec.json 2> gpurun_out/r02n/tdec.err || { echo tdec failed; exit 1; }
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu > gpurun_out/r02n/ue_dl.json 2> gpurun_out/r02n/ue_dl.err || { echo ue_dl failed; exit 1; }
echo rc=0
