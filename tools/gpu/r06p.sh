# round 6 p: the drop-in's resident PDSCH decode on its AVERAGE estimate through the fused equaliser
# (mi355_pdsch_set_ce_invariant): the PDSCH / drop-in / eq_rm GPU suites, then the per-TTI latency A/B
set -o pipefail
OUT=gpurun_out/r06p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_pdsch_gpu.py \
  tests/test_dropin_gpu.py tests/test_eq_rm_gpu.py > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/dropin_ab.sh r06p/ab "MI355_DROPIN_CE_PER_SYMBOL=1" "MI355_DROPIN_CE_PER_SYMBOL=0" 3
