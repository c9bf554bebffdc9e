#!/bin/bash
# r03hm: PDSCH host planning (per-subframe-index map cache, hashed scrambling-sequence cache) -- PDSCH / ue_dl
# parity, host phases, A/B of find_and_decode against the previous build (srsran_amd/lib_var/host0.so)
set -e
OUT=gpurun_out/r03hm
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pdsch_gpu.py tests/test_ue_dl_gpu.py tests/test_uedl_chunks_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
MI355_HOST_PROF=1 timeout -k 10 300 python bench.py --workload ue_dl --steps 4 --warmup 2 --no-cpu --no-waterfall --no-roofline > $OUT/hp.json 2> $OUT/hp.err
for rep in 1 2 3; do
  for lib in srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/host0.so; do
    MI355_LIB=$lib timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/u.json 2> $OUT/u.err
    python -c "import json,sys; u=json.load(open('$OUT/u.json')); print(sys.argv[1], 'ue_dl', u['ms_per_step'], u['crc_ok_tbs'])" $lib >> $OUT/ab.txt
  done
done
echo rc=0
