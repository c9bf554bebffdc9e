#!/bin/bash
# r02e round check on the GPU box: the GPU suite and the default bench.
set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02e/gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02e/bench.json 2> gpurun_out/r02e/bench.err
echo rc=$?
