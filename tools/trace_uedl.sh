#!/bin/bash
# Kernel trace of the find_and_decode workload (run under gpurun from the repo root):
#   tools/trace_uedl.sh <tag> -> gpurun_out/tu_<tag>/ ; summarise with tools/uedl_timeline.py <tag>
set -e
TAG=${1:-cur}
OUT=gpurun_out/tu_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
MI355_HOST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --workload ue_dl --steps 2 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
