#!/bin/bash
# One GPU measurement / closing call (run under gpurun from the repo root):
#     tools/gpu/closing.sh <tag> [phase ...]
# phases (default: suite smoke driver workloads):
#   suite      the whole `-m gpu` suite (the driver's round-end GPU tier)
#   smoke      __graft_entry__.smoke()
#   driver     the driver's literal bench command: python3 bench.py --gpus 1 --steps 20 --warmup 5
#   workloads  ue_dl / tdec / siso_qpsk benches with their MAP-kernel rooflines, drop-in latency loop
#   pmc        MAP-kernel kernel trace + FETCH_SIZE / WRITE_SIZE / SQ passes (tools/pmc_summary.py keys them to the
#              current MAP sources' hash so bench.py's roofline.traffic picks them up)
#   e2estats   rocprofv3 kernel statistics of the default e2e step
# Outputs under gpurun_out/<tag>/.  Every step has its own time limit; the first failure ends the call.
set -e
TAG=${1:?tag}
shift
PHASES=${*:-suite smoke driver workloads}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fail() { rc=$?; echo "$1 rc=$rc"; tail -40 "$2"; exit $rc; }
for ph in $PHASES; do
  echo "== $ph $(date +%T)"
  case $ph in
    suite)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $OUT/suite.log 2>&1 || fail suite $OUT/suite.log
      tail -1 $OUT/suite.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 \
        || fail smoke $OUT/smoke.log
      tail -1 $OUT/smoke.log ;;
    driver)
      timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err \
        || fail driver $OUT/bench.err
      python3 -c "import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); \
print(d['value'], d['ms_per_step'], d['crc_ok_tbs'], d['roofline']['frac'], d['cpu_baseline']['value'])" ;;
    workloads)
      timeout -k 10 300 python3 -u bench.py --workload ue_dl --steps 10 --warmup 3 --no-cpu --no-waterfall \
        > $OUT/ue_dl.json 2> $OUT/ue_dl.err || fail ue_dl $OUT/ue_dl.err
      timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline \
        > $OUT/pdsch_same_box.json 2> $OUT/pdsch_same_box.err || fail pdsch $OUT/pdsch_same_box.err
      timeout -k 10 300 python3 -u bench.py --workload tdec --steps 5 --warmup 2 > $OUT/tdec.json 2> $OUT/tdec.err \
        || fail tdec $OUT/tdec.err
      timeout -k 10 300 python3 -u bench.py --workload siso_qpsk --steps 5 --warmup 2 > $OUT/siso.json \
        2> $OUT/siso.err || fail siso $OUT/siso.err
      timeout -k 10 300 python3 -u tools/dropin_lat.py 1000 > $OUT/dropin_lat.json 2> $OUT/dropin_lat.err \
        || fail dropin_lat $OUT/dropin_lat.err ;;
    pmc)
      B="python3 bench.py --workload tdec --steps 3 --warmup 1 --no-cpu"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B \
        > $OUT/trace.log 2>&1 || fail trace $OUT/trace.log
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B \
        > $OUT/fetch.log 2>&1 || fail fetch $OUT/fetch.log
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B \
        > $OUT/write.log 2>&1 || fail write $OUT/write.log
      timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv \
        -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1 || fail sq $OUT/sq.log ;;
    e2estats)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/e2e -o e2e -- python3 bench.py \
        --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/e2e_tr.json 2> $OUT/e2e_tr.err \
        || fail e2estats $OUT/e2e_tr.err ;;
    *) echo "unknown phase $ph"; exit 2 ;;
  esac
done
echo rc=0
