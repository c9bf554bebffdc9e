#!/bin/bash
# r04g: latency kernel v3 (prefetched blocks, meet point L/3, bitmap fix): DL-SCH tests on both paths, phase probe,
# drop-in latency with the path on / off; pdsch_eq_rm split (MI355_EQRM_DIAG 0/1/2) and its 2-pair-prefetch variant (A/B)
set -e
OUT=gpurun_out/r04g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/dlsch.log 2>&1 || { rc=$?; echo dlsch rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err || { rc=$?; echo probe rc=$rc; [ $rc -eq 1 ] || exit $rc; }
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_off.json 2> $OUT/dropin_lat_off.err
for m in 0 1 2; do
  MI355_EQRM_DIAG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/d$m -o d -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/d$m.json 2> $OUT/d$m.err || { rc=$?; echo d$m rc=$rc; [ $rc -eq 1 ] || exit $rc; }
done
for lib in srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/erpf2.so srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/erpf2.so; do
  MI355_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --no-waterfall --no-roofline > $OUT/ab.json 2> $OUT/ab.err
  python3 -c "import json,sys; r=json.load(open('$OUT/ab.json')); print(sys.argv[1], r['ms_per_step'], r['crc_ok_tbs'])" $lib >> $OUT/ab_erpf.txt
done
echo rc=0
