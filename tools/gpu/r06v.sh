#!/bin/bash
# round 6 v: pdsch_eq_rm's LDS sized by the compact image only for two-layer jobs (SISO regression of r06u) -- PDSCH /
# eq_rm / configs / phy_dl matrix / ue_dl GPU parity, then SISO and the default step, before (head.so) vs after (fix.so)
set -o pipefail
OUT=$PWD/gpurun_out/r06v
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_eq_rm_gpu.py tests/test_pdsch_gpu.py tests/test_configs_gpu.py \
  tests/test_phy_dl_matrix_gpu.py tests/test_ue_dl_gpu.py tests/test_uedl_chunks_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for wl in siso_qpsk pdsch; do
for t in head fix head fix; do
  MI355_LIB=srsran_amd/lib_var/$t.so timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 3 --no-cpu \
    --no-waterfall --no-roofline > $OUT/${wl}_$t.json 2> $OUT/${wl}_$t.err || { tail -20 $OUT/${wl}_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['worker_calls'], d['crc_ok_tbs'])" $OUT/${wl}_$t.json "$wl $t"
done
done
echo rc=0
