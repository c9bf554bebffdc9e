#!/bin/bash
# r04ac: drop-in per-TTI flow traced (kernels + HIP API calls) over 100 TTIs
set -e
OUT=gpurun_out/r04ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --output-format csv -d $OUT/tr -o tr -- python3 tools/dropin_lat.py 100 > $OUT/dropin.json 2> $OUT/dropin.err
echo rc=0
