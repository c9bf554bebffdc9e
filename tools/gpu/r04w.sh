#!/bin/bash
# r04w: pdsch_eq_rm occupancy A/B (workgroups of 512 threads at 6 / 7 / 8 waves per SIMD vs 256 at 5), e2e step and
# eq_rm kernel time on one box
set -e
OUT=gpurun_out/r04w
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base er512w6 er512w7 er512w8; do
    lib=srsran_amd/lib/libsrsran_amd.so; [ $v = base ] || lib=srsran_amd/lib_var/$v.so
    MI355_LIB=$lib timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu --no-waterfall --no-roofline > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err
    python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], r['ms_per_step'], r['crc_ok_tbs'] if 'crc_ok_tbs' in r else '')" $OUT/$v.$rep.json $v
  done
done
MI355_LIB=srsran_amd/lib_var/er512w6.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr6 -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/tr6.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trb -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-waterfall --no-roofline > $OUT/trb.log 2>&1
echo rc=0
