#!/bin/bash
# SQ issue/wait counters of every kernel of the default e2e bench (run under gpurun)
set -e
OUT=gpurun_out/esq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o sq -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log2 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/log3 2>&1
