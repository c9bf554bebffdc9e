#!/bin/bash
# Where the MAP kernel's cycles go (run under gpurun from the repo root):  tools/tdec_stall.sh <tag>
# One --pmc pass per counter group on the turbo-only bench: SQ issue/wait split, L2 hit/miss and memory-side
# requests, and FETCH_SIZE of the loads-only diagnostic build (MI355_TDEC_DIAG=4: every input row read exactly
# once) to calibrate FETCH_SIZE for this kernel's 4-byte-per-lane access pattern.
set -e
TAG=${1:-stall}
OUT=gpurun_out/stall_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 bench.py --workload tdec --steps 2 --warmup 1 --no-cpu"
timeout -k 10 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/tcc -o tcc -- $B > $OUT/tcc.log 2>&1
MI355_TDEC_DIAG=4 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal -o cal -- $B > $OUT/cal.log 2>&1
MI355_TDEC_DIAG=4 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/caltrace -o caltrace -- $B > $OUT/caltrace.log 2>&1
echo done
