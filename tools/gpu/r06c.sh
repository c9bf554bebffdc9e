# round 6 c: (1) pdsch_eq_rm compact vs gather image, one worker (clean kernel durations); (2) the MAP kernel's store
# variants (clone without output stores, non-temporal output / checkpoint stores); (3) the driver's default command
# (roofline, CPU baseline, waterfall with the AVX2-chain CRC parity); (4) the counter list of this part
set -o pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
for c in 0 1; do
  MI355_EQRM_COMPACT=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$c -o run -- python3 bench.py \
    --no-cpu --no-waterfall --no-roofline --workers 1 --steps 10 --warmup 2 > $OUT/prof_c$c.log 2>&1 || exit 1
done
bash tools/gpu/clone_ab.sh r06c_clone srsran_amd/lib_var/base.so srsran_amd/lib_var/clone_noe.so \
  srsran_amd/lib_var/nt_out.so srsran_amd/lib_var/nt_ck.so srsran_amd/lib_var/nt_both.so srsran_amd/lib_var/base.so || exit 1
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
python -c "import json; r=json.load(open('$OUT/bench_default.json')); print(r['value'], r['ms_per_step'], r['crc_ok_tbs']); print(json.dumps(r['e2e_waterfall'])[:3000])"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -c TCC $OUT/avail.txt || true
