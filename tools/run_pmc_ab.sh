#!/bin/bash
# SQ counters of the MAP kernel for library variants: tools/run_pmc_ab.sh <lib>...
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
for lib in "$@"; do
  n=$(basename $lib .so)
  MI355_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcab/$n -o sq -- python3 bench.py --workload tdec --steps 2 --warmup 1 --no-cpu > gpurun_out/pmcab/$n.log 2>&1 || exit 1
done
echo done
