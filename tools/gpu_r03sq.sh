#!/bin/bash
# r03sq: speculative DEC2 half-iterations -- DL-SCH / ue_dl / tdec parity tests, then A/B (MI355_TDEC_SPEC=0/1) of
# the default and ue_dl benches, and the per-dispatch trace of the speculative build
set -e
OUT=gpurun_out/r03sq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dlsch_gpu.py tests/test_uedl_chunks_gpu.py tests/test_tdec_gpu.py tests/test_pdsch_gpu.py tests/test_eq_rm_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
for rep in 1 2; do
  for sp in 1 0; do
    MI355_TDEC_SPEC=$sp timeout -k 10 300 python -u bench.py --no-cpu --no-waterfall --no-roofline > $OUT/p_$sp.json 2> $OUT/p.err
    MI355_TDEC_SPEC=$sp timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > $OUT/u_$sp.json 2> $OUT/u.err
    MI355_TDEC_SPEC=$sp timeout -k 10 300 python -u bench.py --workload siso_qpsk --no-cpu --no-waterfall --no-roofline > $OUT/s_$sp.json 2> $OUT/s.err
    python -c "import json,sys; p=json.load(open('$OUT/p_$sp.json')); u=json.load(open('$OUT/u_$sp.json')); q=json.load(open('$OUT/s_$sp.json')); print('spec', sys.argv[1], 'pdsch', p['ms_per_step'], p['crc_ok_tbs'], 'ue_dl', u['ms_per_step'], u['crc_ok_tbs'], 'siso', q['ms_per_step'], q.get('crc_ok_tbs'))" $sp >> $OUT/ab.txt
  done
done
bash tools/gpu_ktrace.sh sq
echo rc=0
