# round 6: new contract tests + the configs[4] tests, then the configs[4] 1M-subframe rehearsal (8 ranks sharing the
# one GPU over gloo, 3 PHY workers per rank, every payload checked on the GPU)
set -o pipefail
mkdir -p gpurun_out/r06a
(for i in $(seq 1 80); do date +%T >> gpurun_out/r06a/tick; sleep 20; done) &
TK=$!
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_stage_copy_gpu.py tests/test_sync_contracts_gpu.py \
  "tests/test_dropin_gpu.py::test_ctrl_stage_failure_does_not_rerun_estimation" \
  "tests/test_configs_gpu.py::test_config4_total_subframes_two_resident_sets" \
  tests/test_dist_gpu.py > gpurun_out/r06a/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -30 gpurun_out/r06a/tests.log
if [ $rc -eq 0 ]; then
  BENCH_PROGRESS=1 BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 8 \
    --total-subframes 1000000 --resident-gb 6 --warmup 1 > gpurun_out/r06a/bench_c4.json 2> gpurun_out/r06a/bench_c4.err
  rc=$?
  echo "bench rc=$rc"; tail -c 1500 gpurun_out/r06a/bench_c4.err; tail -c 3000 gpurun_out/r06a/bench_c4.json
fi
kill $TK
exit $rc
