#!/bin/bash
# persistent find_and_decode host arrays: ue_dl / control / drop-in GPU tests, A/B, host-phase timings
set -e
OUT=gpurun_out/r03pe
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pdcch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
bash tools/ab_uedl.sh srsran_amd/lib_var/dbuf.so srsran_amd/lib_var/persist.so > $OUT/ab.txt 2>&1
for lib in dbuf persist; do
  MI355_LIB=srsran_amd/lib_var/$lib.so MI355_HOST_PROF=1 timeout -k 10 300 python bench.py --workload ue_dl --steps 4 --warmup 2 --no-cpu --no-waterfall --no-roofline > $OUT/hp_$lib.json 2> $OUT/hp_$lib.err
done
echo rc=0
