#!/bin/bash
# r03c: siso_qpsk workload (configs[2]), default bench with the configs[0] field, ue_dl
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u bench.py --workload siso_qpsk > gpurun_out/r03c/siso.json 2> gpurun_out/r03c/siso.err || { echo siso failed; exit 1; }
timeout -k 10 300 python -u bench.py --no-waterfall > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err || { echo bench failed; exit 1; }
timeout -k 10 300 python -u bench.py --workload ue_dl --no-cpu > gpurun_out/r03c/ue_dl.json 2> gpurun_out/r03c/ue_dl.err || { echo ue_dl failed; exit 1; }
echo rc=0
