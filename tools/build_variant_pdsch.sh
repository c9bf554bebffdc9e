#!/bin/bash
# Build an alternative libsrsran_amd.so whose PDSCH kernels (pdsch_kernels.hip) get extra compile flags, for A/B
# timing (MI355_LIB):  tools/build_variant_pdsch.sh <name> <flags...>  ->  srsran_amd/lib_var/<name>.so
set -e
NAME=$1; shift
cd "$(dirname "$0")/../srsran_amd"
mkdir -p build_var/$NAME lib_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include -ffp-contract=off \
  "$@" -c csrc/pdsch_kernels.hip -o build_var/$NAME/pdsch_kernels.hip.o
OBJS=$(ls build/*.o | grep -v "/pdsch_kernels.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$NAME.so $OBJS build_var/$NAME/pdsch_kernels.hip.o -lpthread
echo lib_var/$NAME.so
