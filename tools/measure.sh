#!/bin/bash
# Round measurement on the GPU box (outputs under gpurun_out/; copy the judged ones to profiles/rN/):
#   A <tag>: the default bench line; the same command under rocprofv3 --kernel-trace --stats (+ the timed window's
#            per-launch averages, tools/rocprof_window.py); the PMC traffic passes over the timed window
#            (tools/pmc_traffic.sh)
#   B <tag>: the other BASELINE configs on the TGN path (mid window)
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
  cd $R && python3 tools/rocprof_window.py gpurun_out/${T}_prof gpurun_out/${T}_bench_under_rocprof.json \
    > gpurun_out/${T}_window_kernel_stats.csv || exit $?
  bash tools/pmc_traffic.sh ${T}
else
  for cfg in "review --dataset tgbl-review --aggr mean" "coin --dataset tgbl-coin" \
             "comment2 --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20"; do
    set -- $cfg
    name=$1; shift
    timeout -k 10 500 python bench.py --model tgn --only --no-cpu-baseline --no-train-loop --no-tcsr "$@" \
      > gpurun_out/${T}_${name}.json 2> gpurun_out/${T}_${name}.err || exit $?
  done
fi
