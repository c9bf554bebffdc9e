#!/bin/bash
# Viterbi branch-metric table + batched decision stores: control-channel GPU tests, then ue_dl A/B vs the
# previous pdcch kernel (run under gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out/vit
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pdcch_gpu.py \
  tests/test_real_signal.py tests/test_real_signal_10m.py tests/test_dropin_gpu.py > gpurun_out/vit/tests.log 2>&1 || { tail -30 gpurun_out/vit/tests.log; exit 1; }
tail -2 gpurun_out/vit/tests.log
A=${A:-tab_pdcch.so}
for lib in srsran_amd/lib_var/$A srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/$A srsran_amd/lib/libsrsran_amd.so; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > gpurun_out/vit/u.json 2>gpurun_out/vit/u.err || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/vit/u.json')); print(sys.argv[1], r['ms_per_step'], r.get('crc_ok_tbs'))" $lib
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vit/prof -o p -- python3 bench.py --workload ue_dl --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > gpurun_out/vit/prof.log 2>&1
