#!/bin/bash
# Build an alternative libsrsran_amd.so where one source file gets extra compile flags, for A/B timing with
# tools/ab_lib.sh (MI355_LIB):  tools/build_variant_src.sh <name> <source.hip> <flags...> -> srsran_amd/lib_var/<name>.so
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../srsran_amd"
mkdir -p build_var/$NAME lib_var
EXTRA=""
case $SRC in pdsch_kernels.hip|pdcch_kernels.hip|enb_dl_kernels.hip|channel_kernels.hip|wiener_kernels.hip) EXTRA="-ffp-contract=off";; esac
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include $EXTRA "$@" \
  -c csrc/$SRC -o build_var/$NAME/$SRC.o
OBJS=$(ls build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$NAME.so $OBJS build_var/$NAME/$SRC.o -lpthread
echo lib_var/$NAME.so
