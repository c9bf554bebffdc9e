#!/bin/bash
# r02f: GPU suite, default bench, MAP kernel profile (PMC keyed to the new sources)
set -o pipefail
mkdir -p gpurun_out/r02f
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02f/gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02f/bench.json 2> gpurun_out/r02f/bench.err && \
bash tools/profile_tdec.sh r02f > gpurun_out/r02f/prof.log 2>&1
echo rc=$?
