#!/bin/bash
# round 6 s: MAP kernel at 3 waves/SIMD where the two-phase beta rebuild (TDEC_NPH 2) fits in 168 VGPRs (DEC2
# instantiations; DEC1 stays at 2) -- parity of the turbo / DL-SCH suites, one-worker kernel statistics of the e2e step
# (kstat_ab) and the tdec workload A/B
set -o pipefail
OUT=gpurun_out/r06s
mkdir -p $OUT
export TMPDIR=/tmp
MI355_LIB=srsran_amd/lib_var/nph2_w3.so timeout -k 10 600 python -u -m pytest tests/test_tdec_gpu.py tests/test_dlsch_gpu.py \
  tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu/kstat_ab.sh r06s_k srsran_amd/lib_var/base.so srsran_amd/lib_var/nph2_w3.so srsran_amd/lib_var/base.so \
  srsran_amd/lib_var/nph2_w3.so || exit 1
bash tools/ab_tdec.sh srsran_amd/lib_var/base.so srsran_amd/lib_var/nph2_w3.so --workload tdec --steps 5 --warmup 2 || exit 1
echo rc=0
