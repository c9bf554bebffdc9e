#!/bin/bash
# Kernel times per subframe at several batch sizes (does a smaller batch's extrinsic stay in the Infinity Cache between
# DEC1 and DEC2?): tools/gpu/batch_ab.sh <tag> <subframes> ...
set -e
OUT=gpurun_out/$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
for b in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b$b -o k -- python3 bench.py --subframes $b --workers 1 --steps 6 --warmup 2 --no-cpu --no-waterfall --no-roofline > $OUT/b$b.json 2> $OUT/b$b.err
  python3 - "$OUT/b$b" "$OUT/b$b.json" "$b" <<'PY'
import csv, glob, json, sys
d, js, b = sys.argv[1:]
b = int(b)
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
r = json.loads(open(js).read().strip().splitlines()[-1])
ks = sorted(((float(x["TotalDurationNs"]), x["Name"].split("(")[0].replace("mi355::", "").replace("void ", "")[:48],
              float(x["AverageNs"]) / 1e3, int(x["Calls"])) for x in csv.DictReader(open(f))), reverse=True)
print(b, "step_ms", r["ms_per_step"], "us per 2048 sf | " + "; ".join(f"{k} {a * 2048 / b:.1f}" for _, k, a, c in ks if a > 20 and 'enb' not in k and 'ofdm_tx' not in k)[:700])
PY
done
echo rc=0
