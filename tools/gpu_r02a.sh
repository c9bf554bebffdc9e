set -o pipefail
mkdir -p gpurun_out/r02a
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/gputest.log 2>&1 && \
timeout -k 10 200 python -u tools/waterfall_sweep.py 512 > gpurun_out/r02a/sweep.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err && \
timeout -k 10 300 python -u bench.py --gpus 1 --total-subframes 8192 --no-cpu > gpurun_out/r02a/bench_total.json 2> gpurun_out/r02a/bench_total.err
echo rc=$?
