#!/bin/bash
# r03b: new config / matrix / chunk tests first, then the full GPU suite and the default bench
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_uedl_chunks_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --durations=0 > gpurun_out/r03b/new.log 2>&1 || { echo new tests failed; exit 1; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b/gputest.log 2>&1 || { echo suite failed; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err || { echo bench failed; exit 1; }
echo rc=0
