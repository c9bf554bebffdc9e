#!/bin/bash
# round 6 z: what the beta-checkpoint traffic costs the MAP schedule in each probe: the bandwidth-only clone with every
# other checkpoint (the traffic of a 16-step spacing) and with none (clone_ab: e2e probe, tdec probe)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/clone_ab.sh r06z srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/ck_half.so srsran_amd/lib_var/no_ck.so \
  srsran_amd/lib/libsrsran_amd.so srsran_amd/lib_var/ck_half.so || exit 1
