#!/bin/bash
# Kernel trace + host phase timing of the default e2e workload (run under gpurun from the repo root):
#   tools/trace_pdsch.sh <tag> -> gpurun_out/tu_<tag>/ ; summarise with tools/uedl_timeline.py <tag> --chunks=1
set -e
TAG=${1:-cur}
OUT=gpurun_out/tu_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MI355_HOST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
