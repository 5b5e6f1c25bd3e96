#!/bin/bash
# round 5: 2-hop tests, comment-shaped 2-hop A/B of the dZr copies, and the three secondary configs over the
# round-4 (start) window
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=$1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "2hop or layers or two or comment" --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
for lib in default $PWD/var/dzr1/libtgnx.so default $PWD/var/dzr1/libtgnx.so; do
  if [ "$lib" = default ]; then unset TGNX_LIB; else export TGNX_LIB=$lib; fi
  timeout -k 10 300 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 10 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(sys.argv[1], d["ms_per_step"], {k: round(v, 1) for k, v in d["kernels_us"].items()})' $lib | tee -a gpurun_out/${T}_dzr_ab.txt || exit 1
done
unset TGNX_LIB
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-review --aggr mean --steps 300 --warmup 30 --window start \
  --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_review_start.json 2>/dev/null || exit 1
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-coin --steps 300 --warmup 30 --window start --no-cpu-baseline \
  --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_coin_start.json 2>/dev/null || exit 1
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --window start \
  --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_comment2_start.json 2>/dev/null || exit 1
