#!/bin/bash
# A variant build of the product library for same-box A/B timing: one source compiled with extra flags, linked with
# the other objects of the current build into srsran_amd/lib_var/<name>.so (load it with MI355_LIB=...).
#   tools/build_var.sh <name> <csrc file> <flags...>     e.g. tools/build_var.sh latd1 tdec_win_lat.hip -DLAT_DIAG=1
set -e
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../srsran_amd"
make -s -j8 lib/libsrsran_amd.so
mkdir -p lib_var /tmp/var_$NAME
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -I../include "$@" -c csrc/$SRC -o /tmp/var_$NAME/$SRC.o
OBJS=$(ls build/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib_var/$NAME.so $OBJS /tmp/var_$NAME/$SRC.o -lpthread
echo lib_var/$NAME.so
