#!/bin/bash
# the drop-in GPU tests alone, repeatedly (intermittent host-crash hunt), with the drop-in's entry-point trace
mkdir -p gpurun_out/dl
for i in 1 2 3 4 5 6 7 8 9 10; do
  SRSLTE_MI355_TRACE=1 timeout -k 10 120 python -u -m pytest tests/test_dropin_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/dl/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  [ $rc -ne 0 ] && exit 1
done
for i in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py tests/test_enb_dl_gpu.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/dl/mix$i.log 2>&1
  rc=$?
  echo "mix $i rc=$rc"
  [ $rc -ne 0 ] && exit 1
done
exit 0
