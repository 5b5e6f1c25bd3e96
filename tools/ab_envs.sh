#!/bin/bash
# Same-box A/B of several environment settings (2 rounds, interleaved), graph-replay bench:
#   [BENCH_ARGS=...] tools/ab_envs.sh <tag> "<ENV=.. ENV2=..>" "-" ...   ("-" = no extra env)
#   -> gpurun_out/<tag>_ab.txt (env, ms_per_step, events/s per run)
tag=$1; shift
out=/root/repo/gpurun_out/${tag}_ab.txt
: > $out
for round in 1 2; do
  for e in "$@"; do
    [ "$e" = "-" ] && envs="" || envs="$e"
    r=$(env $envs timeout -k 10 300 python /root/repo/bench.py --model tgn --only --steps 500 --warmup 50 --no-cpu-baseline --no-train-loop --no-tcsr --no-probe ${BENCH_ARGS:-} 2>/dev/null | grep metric) || exit 1
    echo "$e $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $out
  done
done
