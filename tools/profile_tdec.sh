#!/bin/bash
# Profile the turbo decoder bench on the GPU box (run under gpurun from the repo root).
#   tools/profile_tdec.sh <tag>
# Produces gpurun_out/prof_<tag>/ (kernel trace + stats) and PMC passes (one counter group per pass,
# never combined with tracing domains), then tools/pmc_summary.py writes profiles/<tag>_*.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# kernel trace of the default workload (TM4 ue_dl chain: every kernel), then the turbo-only workload whose
# 65,536-CB MAP launches the PMC passes and the calibration characterise
E="python3 bench.py --steps 3 --warmup 1 --no-cpu"
B="python3 bench.py --workload tdec --steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- $E > $OUT/e2e.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1
# calibration pass: the loads-only diagnostic variant reads a known byte count
MI355_TDEC_DIAG=4 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/calib -o calib -- $B > $OUT/calib.log 2>&1
python3 tools/pmc_summary.py $TAG && mkdir -p gpurun_out/profiles && cp profiles/${TAG}_* profiles/tdec_pmc_traffic.json gpurun_out/profiles/
