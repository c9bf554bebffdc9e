#!/bin/bash
# fused equaliser + LLR + rate dematching (pdsch_eq_rm): parity suites (LLRs via the debug stage, softbuffers vs the
# oracle's rate dematching), then A/B against the two-kernel path and a kernel trace
set -e
OUT=gpurun_out/r03er
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_pdsch_gpu.py tests/test_dlsch_gpu.py tests/test_ue_dl_gpu.py tests/test_dropin_gpu.py tests/test_uedl_chunks_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
for i in 1 2; do
  for v in off on; do
    if [ $v = off ]; then export MI355_NO_EQRM=1; else unset MI355_NO_EQRM; fi
    timeout -k 10 300 python bench.py --no-cpu --no-waterfall --no-roofline > $OUT/b_$v.json 2> $OUT/b_$v.err
    timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/u_$v.json 2> $OUT/u_$v.err
    python -c "import json,sys; p=json.load(open('$OUT/b_$v.json')); u=json.load(open('$OUT/u_$v.json')); print(sys.argv[1], p['ms_per_step'], u['ms_per_step'], p['crc_ok_tbs'], u['crc_ok_tbs'], p.get('payload_checked_tbs'))" $v >> $OUT/ab.txt
  done
done
unset MI355_NO_EQRM
bash tools/trace_pdsch.sh r03er > /dev/null 2>&1
echo rc=0
