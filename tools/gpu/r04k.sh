#!/bin/bash
# r04k: latency kernel SQ counters (instructions, waits) on the probe; find_and_decode kernel timeline + host phases
set -e
OUT=gpurun_out/r04k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq1 -o sq -- python3 tools/lat_probe.py > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d $OUT/sq2 -o sq -- python3 tools/lat_probe.py > $OUT/sq2.log 2>&1
bash tools/trace_uedl.sh r04k
echo rc=0
