# round 6 n: the r06l parity suites again, verbose and with Python's fault handler (r06l: a host segfault at the
# 45th test, which passes alone)
set -o pipefail
OUT=gpurun_out/r06n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -X faulthandler -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eq_rm_gpu.py \
  tests/test_pdsch_gpu.py tests/test_configs_gpu.py tests/test_phy_dl_matrix_gpu.py tests/test_ue_dl_gpu.py \
  tests/test_dlsch_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -60 $OUT/tests.log; exit $rc
