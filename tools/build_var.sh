#!/bin/bash
# Build an A/B variant of the library: tools/build_var.sh NAME [extra hipcc flags...]
# The sources in VAR_SRCS (default: kernels) are recompiled with the extra flags (e.g.
# -DTMED_EXP_...); the other objects come from the in-tree build.
# Output: tendermint-fork_amd/lib_var/NAME/libtmed25519_hip.so
set -eu
name=$1; shift
cd "$(dirname "$0")/../tendermint-fork_amd"
make -s >/dev/null
mkdir -p lib_var/$name /tmp/tmed_var_$name
all="kernels latency tmed_capi signbytes microbench commit keyset merkle zip215 keycache"
objs=""
for s in $all; do
  if [[ " ${VAR_SRCS:-kernels} " == *" $s "* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-value "$@" \
      -c csrc/$s.hip -o /tmp/tmed_var_$name/$s.o
    objs="$objs /tmp/tmed_var_$name/$s.o"
  else
    objs="$objs lib/$s.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o lib_var/$name/libtmed25519_hip.so
echo "built lib_var/$name"
