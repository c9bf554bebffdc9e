# round 6 o: one drop-in TTI loop (tools/dropin_lat.py, 200 TTIs) under a kernel + HIP runtime trace, for the per-TTI
# timeline of launches, copies and host gaps
set -o pipefail
OUT=gpurun_out/r06o
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d $OUT/tr -o t \
  -- python3 -u tools/dropin_lat.py 200 > $OUT/lat.json 2> $OUT/lat.err || { tail -20 $OUT/lat.err; exit 1; }
tail -c 600 $OUT/lat.json
ls $OUT/tr
