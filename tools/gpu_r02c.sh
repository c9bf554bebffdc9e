#!/bin/bash
# r02c round check on the GPU box: GPU suite, default bench, then the MAP-kernel profile (tools/profile_tdec.sh).
set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02c/gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02c/bench.json 2> gpurun_out/r02c/bench.err && \
bash tools/profile_tdec.sh r02c
echo rc=$?
