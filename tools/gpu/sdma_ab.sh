#!/bin/bash
# Worker stalls vs the copy engine: HSA_ENABLE_SDMA=0 (copies as blit kernels on the compute queues) against the default
# (SDMA engines), with simultaneous worker starts (BENCH_STAGGER_MS, default 0 here):  tools/gpu/sdma_ab.sh <tag> [workload]
set -e
OUT=gpurun_out/$1; WL=${2:-pdsch}; mkdir -p $OUT
for rep in 1 2 3; do
  for sd in 1 0; do
    for w in 3 1; do
      f=$OUT/sdma${sd}_w${w}_$rep
      HSA_ENABLE_SDMA=$sd BENCH_STAGGER_MS=${BENCH_STAGGER_MS:-0} timeout -k 10 300 python3 bench.py --workload $WL \
        --workers $w --steps 20 --warmup 5 --no-cpu --no-waterfall --no-roofline > $f.json 2> $f.err \
        || { rc=$?; echo "$f rc=$rc"; tail -20 $f.err; exit $rc; }
      python3 -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['ms_per_step'], r['crc_ok_tbs'], r.get('worker_calls'))" $f.json "$WL sdma=$sd workers=$w"
    done
  done
done
echo rc=0
