# round 6 l: pdsch_eq_rm prologue (descriptor loads in the second wave, first map word before the barrier) vs the
# previous commit (lib_var/prev.so): parity suites, phase profiles, one-worker kernel durations, default bench
set -o pipefail
OUT=gpurun_out/r06l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_eq_rm_gpu.py \
  tests/test_pdsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_ue_dl_gpu.py \
  tests/test_dlsch_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in cur prev; do
  LIBV=""; [ $v != cur ] && LIBV=srsran_amd/lib_var/$v.so
  MI355_LIB=$LIBV timeout -k 10 300 python tools/eqrm_phase.py > $OUT/phase_$v.json 2> $OUT/phase_$v.err || exit 1
  echo "$v $(cat $OUT/phase_$v.json)"
  MI355_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$v -o run -- python3 bench.py \
    --no-cpu --no-waterfall --no-roofline --workers 1 --steps 10 --warmup 2 > $OUT/prof_$v.log 2>&1 || exit 1
done
python tools/kstat_db.py $OUT/prof_*/run_results.db > $OUT/kstat.txt && cat $OUT/kstat.txt
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python -c "import json; r=json.load(open('$OUT/bench_default.json')); print(r['value'], r['ms_per_step'], r['crc_ok_tbs'])"
