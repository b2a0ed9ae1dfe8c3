#!/bin/bash
# Build an A/B variant of the library: tools/build_var.sh NAME [extra hipcc flags...]
# kernels.hip is recompiled with the extra flags (e.g. -DTMED_EXP_...); the other objects
# come from the in-tree build.  Output: tendermint-fork_amd/lib_var/NAME/libtmed25519_hip.so
set -eu
name=$1; shift
cd "$(dirname "$0")/../tendermint-fork_amd"
make -s >/dev/null
mkdir -p lib_var/$name /tmp/tmed_var_$name
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-value "$@" \
  -c csrc/kernels.hip -o /tmp/tmed_var_$name/kernels.o
objs="lib/latency.o lib/tmed_capi.o lib/signbytes.o lib/microbench.o lib/commit.o lib/keyset.o lib/merkle.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC /tmp/tmed_var_$name/kernels.o $objs -o lib_var/$name/libtmed25519_hip.so
echo "built lib_var/$name"
