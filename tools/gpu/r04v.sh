#!/bin/bash
# r04v: configs[2] SISO QPSK kernel trace + host phases (one 8,192-subframe step attributed to kernels); pdsch_eq_rm SQ
# counters (two passes, the e2e bench, the kernel alone by regex)
set -e
OUT=gpurun_out/r04v
mkdir -p $OUT gpurun_out/tu_r04v_siso
export TMPDIR=/tmp
MI355_HOST_PROF=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tu_r04v_siso -o tr -- python3 bench.py --workload siso_qpsk --steps 2 --warmup 1 --no-cpu --no-roofline > gpurun_out/tu_r04v_siso/log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-include-regex pdsch_eq_rm --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/p1 -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/p1.log 2>&1
timeout -s KILL 180 rocprofv3 --kernel-include-regex pdsch_eq_rm --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/p2.log 2>&1
echo rc=0
