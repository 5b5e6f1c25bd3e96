#!/bin/bash
# Round-5 measurement: A <tag> = the default bench line, the same command under rocprofv3 --kernel-trace --stats, and
# the PMC traffic passes (tools/pmc_traffic.sh); B <tag> = the other BASELINE configs on the TGN path.
# Outputs under gpurun_out/ (copy the judged ones to profiles/r5/).
set -o pipefail
R=/root/repo
P=$1; T=${2:-m1}
cd $R
export TMPDIR=/tmp
if [ "$P" = A ]; then
  timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
  cd /tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- \
    python3 $R/bench.py > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_bench_under_rocprof.err || exit $?
  cd $R && bash tools/pmc_traffic.sh ${T}
else
  timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-review --aggr mean --steps 300 --warmup 30 \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_review.json 2> gpurun_out/${T}_review.err || exit $?
  timeout -k 10 500 python bench.py --model tgn --only --dataset tgbl-coin --steps 300 --warmup 30 --no-cpu-baseline \
    --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_coin.json 2> gpurun_out/${T}_coin.err || exit $?
  timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 20 > gpurun_out/${T}_comment2.json 2> gpurun_out/${T}_comment2.err || exit $?
fi
