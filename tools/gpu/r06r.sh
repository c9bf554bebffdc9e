#!/bin/bash
# round 6 r: DEC2 reads its E stream as 16-byte transposed pieces (TDEC_TXE) -- turbo / DL-SCH / configs GPU parity,
# then same-box A/B against the 4-byte build: e2e step + MAP probe + fixed-8, and the tdec workload
set -o pipefail
OUT=gpurun_out/r06r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py tests/test_srslte_tdec_gpu.py \
  tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/ab_lib.sh srsran_amd/lib_var/txe0.so srsran_amd/lib_var/txe1.so || exit 1
bash tools/ab_tdec.sh srsran_amd/lib_var/txe0.so srsran_amd/lib_var/txe1.so --workload tdec --steps 5 --warmup 2 || exit 1
echo rc=0
