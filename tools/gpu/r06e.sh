# round 6 e: compact eq_rm with the interleaved two-layer image (parity suites, phase profile, one-worker kernel
# durations), then the driver's default command
set -o pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_eq_rm_gpu.py \
  tests/test_pdsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_ue_dl_gpu.py \
  tests/test_dlsch_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 0 1; do
  MI355_EQRM_COMPACT=$c timeout -k 10 300 python tools/eqrm_phase.py > $OUT/phase_c$c.json 2> $OUT/phase_c$c.err || exit 1
  echo "compact $c $(cat $OUT/phase_c$c.json)"
  MI355_EQRM_COMPACT=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run -- python3 bench.py \
    --no-cpu --no-waterfall --no-roofline --workers 1 --steps 10 --warmup 2 > $OUT/prof_c$c.log 2>&1 || exit 1
done
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python -c "import json; r=json.load(open('$OUT/bench_default.json')); print(r['value'], r['ms_per_step'], r['crc_ok_tbs']); print(json.dumps(r['e2e_waterfall'])[:2500])"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -c TCC $OUT/avail.txt || true
