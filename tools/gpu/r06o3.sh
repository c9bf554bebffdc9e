#!/bin/bash
# round 6 o3: output-wave handoff variants of the latency turbo kernel (LAT_SPIN_SLEEP, LAT_RING): parity of the DL-SCH
# suite on the default build, then tools/lat_probe.py's phase cycles per variant (two rounds)
set -o pipefail
OUT=$PWD/gpurun_out/r06o3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
for v in s1r2 s0r2 s0r3 s1r3; do
  MI355_LIB=srsran_amd/lib_var/$v.so LAT_PROBE_QUICK=1 timeout -k 10 300 python3 tools/lat_probe.py > $OUT/p_$v.json 2> $OUT/p_$v.err \
    || { tail -20 $OUT/p_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['us_per_call'], d['per_cb_half_it_kcycles'], d['load_kcycles_per_cb'], d['rets'])" $OUT/p_$v.json $v
done
done
echo rc=0
