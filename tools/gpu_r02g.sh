#!/bin/bash
# r02g: GPU suite, default bench, tdec workload bench, e2e kernel stats
set -o pipefail
mkdir -p gpurun_out/r02g
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02g/gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02g/bench.json 2> gpurun_out/r02g/bench.err && \
timeout -k 10 300 python -u bench.py --workload tdec --no-cpu > gpurun_out/r02g/tdec.json 2> gpurun_out/r02g/tdec.err && \
bash tools/e2e_stats.sh r02g
echo rc=$?
