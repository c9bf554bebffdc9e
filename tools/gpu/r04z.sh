#!/bin/bash
# r04z: closing check, second part (after the tdec workload fix): workload tests, tdec / siso_qpsk benches, drop-in
# latency, e2e kernel statistics, trellis-step probe
set -e
OUT=gpurun_out/r04z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bench_workloads_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/wl.log 2>&1 || { rc=$?; echo wl rc=$rc; tail -30 $OUT/wl.log; exit $rc; }
tail -1 $OUT/wl.log
timeout -k 10 300 python3 -u bench.py --workload tdec --steps 5 --warmup 2 --no-cpu > $OUT/tdec.json 2> $OUT/tdec.err
timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 300 python3 -u tools/dropin_lat.py 1000 > $OUT/dropin_lat.json 2> $OUT/dropin_lat.err
timeout -k 10 60 tools/microbench/valu_lat > $OUT/valu_lat.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_tr.json 2> $OUT/e2e_tr.err
echo rc=0
