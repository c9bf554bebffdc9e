#!/bin/bash
# round 6 q: the MAP clone's store attribution with the stored values kept alive (TDEC_CLONE_KEEP): round 5's NO_E clone
# also lost the loads whose only use was the removed stores.  clone_ab (time) and TCC read / write requests per launch.
set -o pipefail
OUT=gpurun_out/r06q
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu/clone_ab.sh r06q_clone srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/clone_noe.so \
  srsran_amd/lib_var/clone_noe_keep.so || exit 1
for v in clone clone_noe clone_noe_keep; do
  lib=srsran_amd/lib/libsrsran_amd.so
  [ $v != clone ] && lib=srsran_amd/lib_var/$v.so
  MI355_LIB=$lib MI355_TDEC_DIAG=20 timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --kernel-include-regex tdec_win_halfit --output-format csv -d $OUT/${v}_p -o c -- python3 tools/map_pmc.py e2e \
    > $OUT/${v}_p.log 2>&1 || exit 1
  echo "done $v"
done
echo rc=0
