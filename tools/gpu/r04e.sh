#!/bin/bash
# r04e: X-schedule latency kernel + fused decision bytes for windows that are not byte-aligned (K = 5312): GPU suite,
# latency-path phase probe, drop-in latency with the path on and off, SISO QPSK bench + trace
set -e
OUT=gpurun_out/r04e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_suite.log 2>&1 || { rc=$?; echo suite rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 200 python3 -u tools/gen_cb_sweep.py > $OUT/gen_cb_sweep.jsonl 2> $OUT/gen_cb_sweep.err || { rc=$?; echo sweep rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err || { rc=$?; echo probe rc=$rc; [ $rc -eq 1 ] || exit $rc; }
MI355_DLSCH_LAT_CBS=512 timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_on.json 2> $OUT/dropin_lat_on.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 500 > $OUT/dropin_lat_off.json 2> $OUT/dropin_lat_off.err
timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/siso -o siso -- python3 bench.py --workload siso_qpsk --steps 3 --warmup 1 --no-cpu --no-roofline > $OUT/siso_tr.json 2> $OUT/siso_tr.err
echo rc=0
