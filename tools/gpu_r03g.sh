#!/bin/bash
# r03g: work-queue blind decoder + swizzled rate-dematcher LDS image: tests, ue_dl bench + trace, e2e bench + trace
set -e
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py tests/test_dlsch_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall > $OUT/bench.json 2> $OUT/bench.err
bash tools/trace_uedl.sh r03g
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e_trace -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $OUT/lds -o lds -- python3 bench.py --workload ue_dl --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/lds.log 2>&1
echo rc=0
