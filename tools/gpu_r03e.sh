#!/bin/bash
# r03e: estimate rows on demand + XCD-chunked estimator / fused equaliser: new test, suite, bench, FETCH of the step
set -e
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ue_dl_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k ce_rows > $OUT/new.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gputest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu --no-waterfall > $OUT/ue_dl.json 2> $OUT/ue_dl.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/e2e_fetch -o fetch -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/e2e_write -o write -- python3 bench.py --steps 1 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_write.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e_trace -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_trace.log 2>&1
echo rc=0
