#!/bin/bash
# Kernel trace of a short default bench run (run under gpurun from the repo root):
#   tools/trace_step.sh <tag>   -> gpurun_out/tr_<tag>/ ; summarise locally with tools/step_timeline.py <tag>
set -e
TAG=${1:-cur}
OUT=gpurun_out/tr_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/log 2>&1
