# round 6 m: the phy_dl matrix alone, verbose, with Python's fault handler (a host segfault in r06l at tm2-4-6)
set -o pipefail
OUT=gpurun_out/r06m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -X faulthandler -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_phy_dl_matrix_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -40 $OUT/tests.log; exit $rc
