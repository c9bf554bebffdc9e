#!/bin/bash
# find_and_decode with chunk decodes left in flight: GPU suite, ue_dl A/B vs the previous build, kernel timeline
# (run under gpurun from the repo root; A = the previous build under srsran_amd/lib_var/)
set -o pipefail
A=${A:-head.so}
mkdir -p gpurun_out/pipe
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pipe/gputest.log 2>&1 || { tail -30 gpurun_out/pipe/gputest.log; exit 1; }
tail -1 gpurun_out/pipe/gputest.log
for lib in srsran_amd/lib_var/$A srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/$A srsran_amd/lib/libsrsran_amd.so; do
  MI355_LIB=$lib timeout -k 10 300 python bench.py --workload ue_dl --no-cpu --no-waterfall --no-roofline > gpurun_out/pipe/u.json 2>gpurun_out/pipe/u.err || exit 1
  python -c "import json,sys; r=json.load(open('gpurun_out/pipe/u.json')); print(sys.argv[1], r['ms_per_step'], r.get('crc_ok_tbs'))" $lib
done
tools/trace_uedl.sh pipe && python3 tools/uedl_timeline.py pipe > gpurun_out/pipe/timeline.txt
