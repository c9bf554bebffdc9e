#!/bin/bash
# host phases + kernel timeline of find_and_decode (current build)
set -e
OUT=gpurun_out/hp
mkdir -p $OUT
export TMPDIR=/tmp
MI355_HOST_PROF=1 timeout -k 10 300 python bench.py --workload ue_dl --steps 4 --warmup 2 --no-cpu --no-waterfall --no-roofline > $OUT/u.json 2> $OUT/u.err
bash tools/trace_uedl.sh hp > /dev/null 2>&1
echo rc=0
