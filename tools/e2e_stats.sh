#!/bin/bash
# Kernel stats of the default e2e bench (run under gpurun):  tools/e2e_stats.sh <tag> -> gpurun_out/es_<tag>/
set -e
TAG=${1:-cur}
OUT=gpurun_out/es_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o es -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
