#!/bin/bash
# A/B graph-replay bench of library variants in one box session (round 5; adds the probed launch times):
#   [BENCH_ARGS="..."] [ROUNDS=2] tools/ab_r5.sh <tag> <lib|default> ...  -> gpurun_out/<tag>_ab.txt
tag=$1; shift
out=/root/repo/gpurun_out/${tag}_ab.txt
: > $out
for round in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset TGNX_LIB; else export TGNX_LIB=$lib; fi
    r=$(timeout -k 10 300 python /root/repo/bench.py --only --steps ${STEPS:-500} --warmup 50 --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 20 ${BENCH_ARGS:-} 2>/dev/null | grep metric) || exit 1
    echo "$lib $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], {k: round(v, 2) for k, v in d["kernels_us"].items()})')" | tee -a $out
  done
done
