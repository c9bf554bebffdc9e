#!/bin/bash
# round 6 w: one-worker SISO kernel statistics, head.so vs fix.so (pdsch_eq_rm<2,0> LDS sizing)
set -o pipefail
export TMPDIR=/tmp
WL=siso_qpsk bash tools/gpu/kstat_ab.sh r06w_k srsran_amd/lib_var/head.so srsran_amd/lib_var/fix.so srsran_amd/lib_var/head.so srsran_amd/lib_var/fix.so | cut -c1-400 || exit 1
