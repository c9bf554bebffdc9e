#!/bin/bash
# r03o: CB CRC check fused into the MAP kernel's decision-byte epilogue + in-order staging uploads: DL-SCH / PDSCH /
# turbo / ue_dl / control / drop-in tests, pdsch + ue_dl bench, ue_dl timeline
set -e
OUT=gpurun_out/r03o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dlsch_gpu.py tests/test_pdsch_gpu.py tests/test_tdec_gpu.py tests/test_srslte_tdec_gpu.py tests/test_ue_dl_gpu.py tests/test_uedl_chunks_gpu.py tests/test_pdcch_gpu.py tests/test_dropin_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/pdsch.json 2> $OUT/pdsch.err
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/ue_dl.json 2> $OUT/ue_dl.err
bash tools/trace_uedl.sh r03o
echo rc=0
