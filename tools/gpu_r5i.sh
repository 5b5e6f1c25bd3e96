#!/bin/bash
# round 5: comment-shaped 2-hop B = 600 (start window) A/B: this build against the round-4 final library
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lib in default $PWD/var/r4/libtgnx.so default $PWD/var/r4/libtgnx.so; do
  if [ "$lib" = default ]; then unset TGNX_LIB; else export TGNX_LIB=$lib; fi
  timeout -k 10 300 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --window start \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 10 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], d["config"]["sampled_edges_per_step"], {k: round(v, 1) for k, v in d["kernels_us"].items()})' $lib | tee -a gpurun_out/${1}_ab.txt || exit 1
done
