#!/bin/bash
# Clock-independent A/B of the C2 kernels: one rocprofv3 --pmc pass per variant (VALU instructions,
# wave cycles, GPU-active cycles per dispatch), summarized by tools/pmc_summary.py.  The live
# bench figures move with the box's clock (the measured mad peak varies +-3 % between runs on one
# box); cycles per dispatch do not.  Arguments as tools/ab.sh: cur, env:VAR=value[,..], lib_var NAME.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
mkdir -p $OUT
for v in "$@"; do
  envs=""
  case $v in
    env:*) lib=tendermint-fork_amd/lib/libtmed25519_hip.so; envs=${v#env:};;
    cur) lib=tendermint-fork_amd/lib/libtmed25519_hip.so;;
    *) lib=tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so;;
  esac
  tag=$(echo "$v" | tr ':=,' '___')
  env ${envs//,/ } TMED_LIB=$PWD/$lib timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_INT64 SQ_WAVES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d $PWD/$OUT/$tag -o run -- python3 $PWD/bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-peak --no-c1 ${PMC_BENCH_ARGS:---no-keyset} --no-c4 --no-c5 --no-zip215 > $OUT/$tag.log 2>&1 || exit $?
  python3 tools/pmc_summary.py $OUT/$tag.json $OUT/$tag > /dev/null 2>&1
  python3 - "$OUT/$tag.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k in ("verify_main_hs_kernel", "verify_prep_kernel", "verify_prep_r_kernel", "verify_keyset_prep_kernel", "verify_keyset_main_kernel"):
    r = d.get(k)
    if r:
        print(sys.argv[2], k, "gpu_cycles/8 %.0f" % (r["GRBM_GUI_ACTIVE"] / 8), "valu/wave %.0f" % r["valu_insts_per_wave"],
              "int64/wave %.0f" % (r["SQ_INSTS_VALU_INT64"] / r["SQ_WAVES"]) if "SQ_WAVES" in r else "")
PY
done
