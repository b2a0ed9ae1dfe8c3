#!/bin/bash
# Build an A/B variant of the engine library: tools/build_ab.sh TAG "EXTRA HIPFLAGS" [sources...]
# Recompiles the named csrc sources (default: kernels latency) with the extra flags, reuses the
# other objects of the main build, and links tendermint-fork_amd/lib/ab/libtmed_TAG.so (loaded
# through TMED_LIB by the A/B tools).
set -eu
cd "$(dirname "$0")/../tendermint-fork_amd"
TAG=$1; EXTRA=$2; shift 2
SRCS=${*:-kernels latency}
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result"
OBJ=lib/ab/obj_$TAG
mkdir -p $OBJ
objs=""
for o in kernels latency tmed_capi signbytes microbench commit keyset merkle zip215 keycache; do
  if [[ " $SRCS " == *" $o "* ]]; then
    /opt/rocm/bin/hipcc $HIPFLAGS $EXTRA -c csrc/$o.hip -o $OBJ/$o.o
    objs="$objs $OBJ/$o.o"
  else
    objs="$objs lib/$o.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o lib/ab/libtmed_$TAG.so
rm -rf $OBJ
echo lib/ab/libtmed_$TAG.so
