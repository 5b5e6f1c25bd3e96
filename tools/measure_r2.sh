#!/bin/bash
# Round-2 measurement: default bench line, the same command under rocprofv3 --kernel-trace --stats, and
# the other BASELINE configs on the TGN path.  Outputs under gpurun_out/ (copy the judged ones to profiles/).
set -o pipefail
R=/root/repo
cd $R
timeout -k 10 900 python bench.py > gpurun_out/m2_bench.json 2> gpurun_out/m2_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/m2_prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/m2_bench_under_rocprof.json 2> $R/gpurun_out/m2_bench_under_rocprof.err || exit $?
cd $R
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-review --aggr mean --steps 300 --warmup 30 \
  --no-cpu-baseline --probe-steps 20 > gpurun_out/m2_review.json 2> gpurun_out/m2_review.err || exit $?
timeout -k 10 500 python bench.py --model tgn --only --dataset tgbl-coin --steps 300 --warmup 30 --no-cpu-baseline \
  --probe-steps 20 > gpurun_out/m2_coin.json 2> gpurun_out/m2_coin.err || exit $?
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 \
  --no-cpu-baseline --probe-steps 20 > gpurun_out/m2_comment2.json 2> gpurun_out/m2_comment2.err
cd $R && bash tools/pmc_traffic.sh m2
