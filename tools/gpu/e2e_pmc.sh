#!/bin/bash
# Per-kernel PMC passes of the default e2e step (run under gpurun): tools/gpu/e2e_pmc.sh <tag>
# -> gpurun_out/pmc_<tag>/{trace,fetch,write,sq,lds}; summarise with tools/e2e_pmc_summary.py-style readers.
set -e
TAG=${1:?tag}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
E="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-roofline --no-waterfall"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $E > $OUT/trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $E > $OUT/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $E > $OUT/write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o sq -- $E > $OUT/sq.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $OUT/lds -o lds -- $E > $OUT/lds.log 2>&1
echo rc=0
