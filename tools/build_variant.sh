#!/bin/bash
# Build an alternative libsrsran_amd.so whose turbo-decoder kernels get extra compile flags, for A/B timing with
# tools/ab_tdec.sh (MI355_LIB):  tools/build_variant.sh <name> <flags...>  ->  srsran_amd/lib_var/<name>.so
set -e
NAME=$1; shift
cd "$(dirname "$0")/../srsran_amd"
mkdir -p build_var/$NAME lib_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" \
  -c csrc/tdec_kernels.hip -o build_var/$NAME/tdec_kernels.hip.o
OBJS=$(ls build/*.o | grep -v "/tdec_kernels.hip.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$NAME.so $OBJS build_var/$NAME/tdec_kernels.hip.o -lpthread
echo lib_var/$NAME.so
