#!/bin/bash
# MAP kernel 16-byte transposed loads: microbenchmark, turbo/DL-SCH GPU parity, then A/B in the bench
set -o pipefail
mkdir -p gpurun_out/tx
timeout -k 10 120 tools/microbench/map_overlap 65536 > gpurun_out/tx/mb.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_tdec_gpu.py tests/test_srslte_tdec_gpu.py tests/test_dlsch_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tx/test.log 2>&1 && \
for tx in 1 0 1 0; do MI355_TDEC_TX=$tx timeout -k 10 300 python bench.py --no-cpu --no-waterfall > gpurun_out/tx/b$tx.json 2>gpurun_out/tx/b$tx.err || exit 1; python -c "import json,sys; r=json.load(open(sys.argv[1])); print('tx', sys.argv[2], r['ms_per_step'], r['roofline']['avg_launch_ms'], r['decoder_bound_fixed8']['ms'] if 'decoder_bound_fixed8' in r else '')" gpurun_out/tx/b$tx.json $tx; done
echo rc=$?
