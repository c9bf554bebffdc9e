# round 6 b: eq_rm compact image (parity suites, then same-box A/B of MI355_EQRM_COMPACT), then the MAP kernel's
# deferred output flush (clone + real kernel, A/B against the base build)
set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_eq_rm_gpu.py \
  tests/test_pdsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_ue_dl_gpu.py \
  tests/test_dlsch_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for c in 0 1; do
    MI355_EQRM_COMPACT=$c timeout -k 10 300 python bench.py --no-cpu --no-waterfall --steps 10 --warmup 2 > $OUT/eqrm_c$c.json 2> $OUT/eqrm_c$c.err || exit 1
    python -c "import json,sys; r=json.load(open(sys.argv[1])); print('compact', sys.argv[2], r['ms_per_step'], r['crc_ok_tbs'], r.get('stage_ms'))" $OUT/eqrm_c$c.json $c
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for c in 0 1; do
  MI355_EQRM_COMPACT=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run -- python3 bench.py \
    --no-cpu --no-waterfall --no-roofline --steps 10 --warmup 2 > $OUT/prof_c$c.log 2>&1 || exit 1
done
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; grep -E "pdsch_eq_rm|tdec_win_halfit" "$f" | cut -c1-200; done
bash tools/gpu/clone_ab.sh r06b_clone srsran_amd/lib_var/base.so srsran_amd/lib_var/defer.so srsran_amd/lib_var/defer_fpf3.so srsran_amd/lib_var/base.so srsran_amd/lib_var/defer.so
