#!/bin/bash
# r03h (round-3 head, same passes as r03d): counter list, FETCH/WRITE calibration microbenchmark, LDS bank-conflict counters of the find_and_decode
# workload (MAP, rate dematcher, blind decoder), per-kernel FETCH/WRITE of the default e2e step
set -e
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o cal_fetch -- ./tools/microbench/fetch_calib > $OUT/cal_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o cal_write -- ./tools/microbench/fetch_calib > $OUT/cal_write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/lds -o lds -- python3 bench.py --workload ue_dl --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/lds.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/e2e_fetch -o fetch -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/e2e_write -o write -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_write.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e_trace -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_trace.log 2>&1
python3 tools/r03_pmc_summary.py r03h && mkdir -p gpurun_out/profiles && cp profiles/r03h_pmc.json gpurun_out/profiles/
echo rc=0
