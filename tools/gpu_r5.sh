#!/bin/bash
# On the GPU box (round 5): a pytest run of the given test selection, output streamed to a log under gpurun_out/.
#   tools/gpu_r5.sh <tag> <timeout s> <pytest args...>   -> gpurun_out/<tag>_tests.log
tag=$1; lim=$2; shift 2
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 "$lim" python -u -m pytest "$@" -m gpu -x -v -s --timeout 900 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || grep -E "Error|assert|FAILED" gpurun_out/${tag}_tests.log | head -30
exit $rc
