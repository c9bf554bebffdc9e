# round 6 g: the MAP kernel's output / checkpoint stores with an explicit cache policy (buffer stores: plain, sc1
# write-through), real kernel and clone, then the write-path counters of plain vs sc1 output stores
set -o pipefail
OUT=gpurun_out/r06g
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu/clone_ab.sh r06g_clone srsran_amd/lib_var/base.so srsran_amd/lib_var/out_buf0.so \
  srsran_amd/lib_var/out_sc1.so srsran_amd/lib_var/both_sc1.so srsran_amd/lib_var/base.so || exit 1
P1=TCC_EA0_WRREQ_sum,TCC_EA0_RDREQ_sum,TCC_EA0_RDREQ_128B_sum,TCC_EA0_RDREQ_64B_sum
for v in base out_sc1 both_sc1; do
  MI355_LIB=srsran_amd/lib_var/$v.so timeout -s KILL 240 rocprofv3 --pmc $(echo $P1 | tr ',' ' ') \
    --kernel-include-regex tdec_win_halfit --output-format csv -d $OUT/${v}_p1 -o c -- python3 tools/map_pmc.py e2e \
    > $OUT/${v}_p1.log 2>&1 || exit 1
  echo "done $v"
done
echo rc=0
