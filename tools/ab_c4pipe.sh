#!/bin/bash
# A/B of blocksync-seam host settings on one box, alternating rounds: bench_commits.py --config c4
# with the seam trace (per-batch host phases, copy-in and kernel times).  Each argument is one
# variant, a space-separated list of VAR=value settings (e.g. "TMED_PIPE_SLOTS=2 TMED_HOST_NUMA=0").
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/c4ab
mkdir -p $OUT
for r in $(seq 1 ${ROUNDS:-2}); do
  v=0
  for cfg in "$@"; do
    v=$((v + 1))
    env $cfg TMED_TRACE=1 timeout -k 10 200 python bench_commits.py --config c4 --blocks ${BLOCKS:-4000} --no-cpu \
      > $OUT/v$v.$r.jsonl 2> $OUT/v$v.$r.err || exit $?
    echo "$r [$cfg] $(tail -1 $OUT/v$v.$r.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,1), d["host_phase_per_batch_ms"][0])')" | tee -a $OUT/ab.txt
  done
done
