# round 6 f: (1) pdsch_eq_rm occupancy / pairs-in-flight variants (one worker, kernel durations); (2) the MAP kernel's
# write path on the counters: real kernel, bandwidth-only clone, clone without the output stores (tools/map_pmc.py e2e)
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
WL=pdsch bash tools/gpu/kstat_ab.sh r06f_er srsran_amd/lib_var/er_base.so srsran_amd/lib_var/er_pf2.so \
  srsran_amd/lib_var/er_w4.so srsran_amd/lib_var/er_pf2_w4.so srsran_amd/lib_var/er_base.so | grep -v "^rc=" || exit 1
P1=TCC_EA0_WRREQ_sum,TCC_EA0_WRREQ_64B_sum,TCC_EA0_WRREQ_STALL_sum,TCC_TOO_MANY_EA_WRREQS_STALL_sum
P2=TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum,TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum,TCC_TAG_STALL_sum,TCC_EA0_RDREQ_sum
for v in real clone clone_noe; do
  lib=srsran_amd/lib/libsrsran_amd.so; diag=0
  [ $v = clone ] && diag=20
  [ $v = clone_noe ] && diag=20 && lib=srsran_amd/lib_var/clone_noe.so
  for p in 1 2; do
    eval PM=\$P$p
    MI355_LIB=$lib MI355_TDEC_DIAG=$diag timeout -s KILL 240 rocprofv3 --pmc $(echo $PM | tr ',' ' ') \
      --kernel-include-regex tdec_win_halfit --output-format csv -d $OUT/${v}_p$p -o c -- python3 tools/map_pmc.py e2e \
      > $OUT/${v}_p$p.log 2>&1 || exit 1
  done
  MI355_LIB=$lib MI355_TDEC_DIAG=$diag timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/${v}_kt -o k -- python3 tools/map_pmc.py e2e > $OUT/${v}_kt.log 2>&1 || exit 1
  echo "done $v"
done
echo rc=0
