mkdir -p gpurun_out/c4a
(for i in $(seq 1 60); do date +%T >> gpurun_out/c4a/tick; sleep 20; done) &
TK=$!
BENCH_DIST_BACKEND=gloo BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 8 --total-subframes 1000000 --resident-gb 6 --warmup 1 > gpurun_out/c4a/bench.log 2>&1
rc=$?
kill $TK
echo rc=$rc
tail -c 3000 gpurun_out/c4a/bench.log
exit $rc
