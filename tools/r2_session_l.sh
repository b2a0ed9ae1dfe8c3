#!/bin/bash
# Kernel-trace A/B of library variants (rocprofv3 average durations of the C2 kernels over
# STEPS calls each), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r2l
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for v in ${VARIANTS:-cur}; do
    if [ "$v" = cur ]; then lib=$R/tendermint-fork_amd/lib/libtmed25519_hip.so; else lib=$R/tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
    TMED_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v.$r -o run --output-format csv -- python3 $R/bench.py --steps ${STEPS:-30} --warmup 1 --no-cpu-baseline --no-keyset --no-c1 --no-peak > $OUT/$v.$r.log 2>&1 || exit $?
    python3 - $OUT/$v.$r <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
d = {r["Name"].split("(")[0].split("::")[-1]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
print(sys.argv[1].split("/")[-1], {k: round(d[k], 1) for k in ("verify_prep_kernel", "verify_prep_r_kernel", "verify_main_hs_kernel") if k in d})
PY
  done
done
