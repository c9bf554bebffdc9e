#!/bin/bash
# dlsch + drop-in GPU tests repeatedly with the drop-in entry-point trace (intermittent host-crash hunt)
mkdir -p gpurun_out/dl
for i in 1 2 3 4 5 6 7 8; do
  SRSLTE_MI355_TRACE=1 timeout -k 10 200 python -X faulthandler -u -m pytest tests/test_dlsch_gpu.py tests/test_dropin_gpu.py -x -v -s --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/dl/tmix$i.log 2>&1
  rc=$?
  echo "tmix $i rc=$rc"
  [ $rc -ne 0 ] && exit 1
done
exit 0
