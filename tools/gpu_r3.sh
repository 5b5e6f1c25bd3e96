#!/bin/bash
# On the GPU box, one round-3 iteration: GPU tests (all, or a pytest -k subset), then bench lines of the
# BASELINE configs on the TGN path with their per-launch times.
#   tools/gpu_r3.sh <tag> [pytest -k expr | -] [wiki review coin comment2 ...]
#   -> gpurun_out/<tag>_tests.log, gpurun_out/<tag>_<config>.json
tag=${1:-r3}; kexpr=${2:--}; shift 2 2>/dev/null
cfgs=${*:-wiki review coin comment2}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ "$kexpr" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr" > gpurun_out/${tag}_tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
fi
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
for cfg in $cfgs; do
  case $cfg in
    wiki) args="--steps 500 --warmup 50" ;;
    review) args="--dataset tgbl-review --aggr mean --steps 300 --warmup 30" ;;
    coin) args="--dataset tgbl-coin --steps 300 --warmup 30" ;;
    comment2) args="--dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20" ;;
    *) echo "unknown config $cfg"; exit 2 ;;
  esac
  timeout -k 10 400 python bench.py --model tgn --only --no-cpu-baseline --probe-steps 20 $args \
    > gpurun_out/${tag}_${cfg}.json 2> gpurun_out/${tag}_${cfg}.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_${cfg}.json')); print('$cfg', d['value'], d['ms_per_step'], {k: round(v,1) for k,v in d['kernels_us'].items()})"
done
