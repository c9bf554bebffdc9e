#!/bin/bash
# the GPU suite twice in a row (intermittent-failure check), then the default bench
set -o pipefail
mkdir -p gpurun_out/fl
for i in 1 2; do
  timeout -k 10 500 python -X faulthandler -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/fl/gputest$i.log 2>&1 || { echo "suite $i rc=$?"; exit 1; }
done
timeout -k 10 300 python -u bench.py > gpurun_out/fl/bench.json 2> gpurun_out/fl/bench.err
echo rc=$?
