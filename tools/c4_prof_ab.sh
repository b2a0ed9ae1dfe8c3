set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/t
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t/slot.log 2>&1; echo tests rc=$?
cd /tmp && export TMPDIR=/tmp
for v in cur noslot; do
  if [ $v = cur ]; then L=$GRAFT_REPO_ROOT/tendermint-fork_amd/lib/libtmed25519_hip.so; else L=$GRAFT_REPO_ROOT/tendermint-fork_amd/lib_var/$v/libtmed25519_hip.so; fi
  TMED_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c4prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench_commits.py --config c4 --blocks 4000 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/c4prof_$v.log 2>&1 || exit 1
  echo "$v done"
done
