#!/bin/bash
# A/B graph-replay bench of library variants in one box session:
#   [MODEL=tgnn] [BENCH_ARGS="--dataset tgbl-review --aggr mean"] tools/ab_bench.sh <tag> <lib|default> ...  -> gpurun_out/<tag>_ab.txt (ms_per_step per run, 2 rounds)
tag=$1; shift
out=/root/repo/gpurun_out/${tag}_ab.txt
: > $out
for round in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset TGNX_LIB; else export TGNX_LIB=$lib; fi
    r=$(timeout -k 10 300 python /root/repo/bench.py --model ${MODEL:-tgn} --only --steps 500 --warmup 50 --no-cpu-baseline --no-train-loop --no-tcsr --no-probe ${BENCH_ARGS:-} 2>/dev/null | grep metric) || exit 1
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')" >> $out
  done
done
