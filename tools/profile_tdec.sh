#!/bin/bash
# Profile the turbo decoder on the GPU box (run under gpurun from the repo root):  tools/profile_tdec.sh <tag>
# Produces gpurun_out/prof_<tag>/ (kernel trace + stats of the default e2e bench and of the turbo-only bench) and
# one PMC pass per counter group (never combined with tracing domains), then tools/pmc_summary.py writes
# profiles/<tag>_* and profiles/r02_tdec_pmc.json.  Every step has its own time limit; the first failure ends it.
set -e
TAG=${1:-r02}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
E="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline"
B="python3 bench.py --workload tdec --steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- $E > $OUT/e2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1
python3 tools/pmc_summary.py $TAG
mkdir -p gpurun_out/profiles && cp profiles/${TAG}_* profiles/r02_tdec_pmc.json gpurun_out/profiles/
