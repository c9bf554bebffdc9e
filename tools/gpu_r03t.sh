#!/bin/bash
# r03t: e2e (pdsch workload) kernel timeline + host phases
set -e
export TMPDIR=/tmp
bash tools/trace_pdsch.sh r03t
echo rc=0
