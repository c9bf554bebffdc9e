#!/bin/bash
# r04f: pdsch_eq_rm split -- kernel time with its rate dematching skipped (MI355_EQRM_DIAG=1) and with its equaliser
# skipped (=2) against the full kernel; measurement only (the diagnostic runs decode nothing)
set -e
OUT=gpurun_out/r04f
mkdir -p $OUT
export TMPDIR=/tmp
for m in 0 1 2; do
  MI355_EQRM_DIAG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/d$m -o d -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/d$m.json 2> $OUT/d$m.err || { rc=$?; echo d$m rc=$rc; [ $rc -eq 1 ] || exit $rc; }
done
echo rc=0
