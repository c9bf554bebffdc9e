# round 6 d: (1) MAP workspace address aliasing test (gaps between the a-priori / extrinsic / decision arrays);
# (2) pdsch_eq_rm phase profile, compact image vs gather image; (3) the driver's default command; (4) counter list
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
export TMPDIR=/tmp
for pad in 0 4352 67584 1060864 0; do
  MI355_TDEC_WS_PAD=$pad timeout -k 10 300 python bench.py --no-cpu --no-waterfall --steps 3 --warmup 1 > $OUT/pad_$pad.json 2> $OUT/pad_$pad.err || exit 1
  python -c "import json,sys; r=json.load(open(sys.argv[1]))['roofline']; print('pad', sys.argv[2], r['avg_launch_ms'], r.get('schedule_clone_ms'))" $OUT/pad_$pad.json $pad
done
for c in 0 1 0 1; do
  MI355_EQRM_COMPACT=$c timeout -k 10 300 python tools/eqrm_phase.py > $OUT/phase_c$c.json 2> $OUT/phase_c$c.err || exit 1
  echo "compact $c $(cat $OUT/phase_c$c.json)"
done
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python -c "import json; r=json.load(open('$OUT/bench_default.json')); print(r['value'], r['ms_per_step'], r['crc_ok_tbs']); print(json.dumps(r['e2e_waterfall'])[:2500])"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -c TCC $OUT/avail.txt || true
