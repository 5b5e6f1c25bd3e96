#!/bin/bash
# round 5: full GPU suite, then comment-shaped 2-hop B = 600 with the predictor's multi-event workgroups against one
# event per workgroup (TGNX_PRED_GROUPS large), and the wiki step
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for g in default 100000 default 100000; do
  if [ "$g" = default ]; then unset TGNX_PRED_GROUPS; else export TGNX_PRED_GROUPS=$g; fi
  timeout -k 10 300 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --window start \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 10 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("groups", sys.argv[1], d["ms_per_step"], {k: round(v, 1) for k, v in d["kernels_us"].items()})' $g | tee -a gpurun_out/${T}_ab.txt || exit 1
done
unset TGNX_PRED_GROUPS
STEPS=500 ROUNDS=1 tools/ab_r5.sh ${T}w default
