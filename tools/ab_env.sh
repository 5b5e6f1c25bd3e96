#!/bin/bash
# Same-box A/B of environment settings on one bench configuration, R rounds (default 3), interleaved:
#   tools/ab_env.sh <tag> "<env A>" "<env B>" [bench args...]   (env "-" = none)
#   -> gpurun_out/<tag>_ab.txt: one line per run: env, ms_per_step, events/s
tag=$1; A=$2; B=$3; shift 3
cd "$(dirname "$0")/.."
out=gpurun_out/${tag}_ab.txt
: > $out
for round in $(seq ${ROUNDS:-3}); do
  for e in "$A" "$B"; do
    [ "$e" = "-" ] && envs="" || envs="$e"
    r=$(env $envs timeout -k 10 300 python bench.py --model tgn --only --no-cpu-baseline --no-train-loop --no-tcsr --no-probe "$@" 2>/dev/null | grep metric) || exit 1
    echo "$e $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $out
  done
done
cat $out
