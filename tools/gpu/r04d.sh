#!/bin/bash
# r04d: latency-path phase probe; e2e kernel trace (step time 3.56 -> 4.20 ms between r04b and r04c); SISO QPSK bench
# with the deduplicated PDCCH hit records
set -e
OUT=gpurun_out/r04d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/lat_probe.py > $OUT/lat_probe.jsonl 2> $OUT/lat_probe.err || { rc=$?; echo probe rc=$rc; [ $rc -eq 1 ] || exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e.json 2> $OUT/e2e.err
timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/siso.json 2> $OUT/siso.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/siso -o siso -- python3 bench.py --workload siso_qpsk --steps 3 --warmup 1 --no-cpu --no-roofline > $OUT/siso_tr.json 2> $OUT/siso_tr.err
echo rc=0
