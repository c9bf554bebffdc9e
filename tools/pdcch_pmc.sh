#!/bin/bash
# SQ counters of the control-channel kernels in the find_and_decode workload (run under gpurun)
set -e
OUT=gpurun_out/pdpmc
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $OUT/sq -o sq -- python3 bench.py --workload ue_dl --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
