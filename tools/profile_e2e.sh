#!/bin/bash
# Per-kernel PMC passes over the default (TM4 ue_dl) bench workload (run under gpurun from the repo root):
#   tools/profile_e2e.sh <tag>  -> gpurun_out/pmc_<tag>/ ; summarise locally: python3 tools/e2e_pmc_summary.py <tag>
# One counter group per pass, never combined with tracing domains.
set -e
TAG=${1:-cur}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
E="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-roofline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $E > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $E > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $E > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o sq -- $E > $OUT/sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o tcc -- $E > $OUT/tcc.log 2>&1
