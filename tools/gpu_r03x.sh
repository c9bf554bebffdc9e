#!/bin/bash
# r03x: persistent MAP grid (2 blocks per CU) for the DL-SCH's half-iterations >= 2: DL-SCH / PDSCH / turbo / ue_dl /
# config / drop-in tests, A/B e2e + ue_dl, waterfall (same CRC-ok count), ue_dl timeline
set -e
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dlsch_gpu.py tests/test_pdsch_gpu.py tests/test_tdec_gpu.py tests/test_srslte_tdec_gpu.py tests/test_ue_dl_gpu.py tests/test_uedl_chunks_gpu.py tests/test_configs_gpu.py tests/test_dropin_gpu.py tests/test_phy_dl_matrix_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/prev.so srsran_amd/lib_var/new.so > $OUT/ab.txt 2>&1
timeout -k 10 300 python -u bench.py --no-cpu --no-roofline > $OUT/bench_wf.json 2> $OUT/bench_wf.err
bash tools/trace_uedl.sh r03x
echo rc=0
