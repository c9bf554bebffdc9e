set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_pdcch_gpu.py tests/test_real_signal.py tests/test_dropin_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fad.log 2>&1 && \
MI355_HOST_PROF=1 timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall --steps 5 > gpurun_out/uedl.json 2> gpurun_out/uedl.err
echo rc=$?
