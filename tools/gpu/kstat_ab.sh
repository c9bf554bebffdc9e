#!/bin/bash
# Kernel-time A/B of library builds on one box (run under gpurun): tools/gpu/kstat_ab.sh <tag> <lib.so> ...
# rocprofv3 kernel statistics of the default e2e step (3 steps) per library; prints per library the step time and the
# average duration of every kernel above 20 us.
set -e
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); n=$(basename $lib .so)_$i
  MI355_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o k -- python3 bench.py --workload ${WL:-pdsch} --workers 1 --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/$n.json 2> $OUT/$n.err
  python3 - "$OUT/$n" "$OUT/$n.json" "$n" <<'PY'
import csv, glob, json, sys
d, js, n = sys.argv[1:]
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
r = json.loads(open(js).read().strip().splitlines()[-1])
ks = sorted(((float(x["TotalDurationNs"]), x["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("mi355::", "").replace("void ", "")[:48],
              float(x["AverageNs"]) / 1e3, int(x["Calls"])) for x in csv.DictReader(open(f))), reverse=True)
print(n, "step_ms", r["ms_per_step"], "| " + "; ".join(f"{k} {a:.1f}us x{c}" for _, k, a, c in ks if a > 20)[:900])
PY
done
echo rc=0
