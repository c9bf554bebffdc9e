#!/bin/bash
# r04p: SQ counters of the latency kernel (two passes over the quick probe)
set -e
OUT=gpurun_out/r04p
mkdir -p $OUT
export TMPDIR=/tmp LAT_PROBE_QUICK=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL --output-format csv -d $OUT/p1 -o p -- python3 tools/lat_probe.py > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT --output-format csv -d $OUT/p2 -o p -- python3 tools/lat_probe.py > $OUT/p2.log 2>&1
echo rc=0
