#!/bin/bash
# TGNN B = 200 kernel stats (graph replay, timed window) with the folded-Adam step
set -o pipefail
R=/root/repo
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${1:-r6m}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_tgnn_prof -o run -- \
  python3 $R/bench.py --model tgnn --only --no-cpu-baseline --no-train-loop --no-tcsr --no-config1 \
  > $R/gpurun_out/${T}_tgnn_bench.json 2> $R/gpurun_out/${T}_tgnn_bench.err || exit $?
cd $R && python3 tools/rocprof_window.py gpurun_out/${T}_tgnn_prof gpurun_out/${T}_tgnn_bench.json \
  > gpurun_out/${T}_tgnn_window_kernel_stats.csv || exit $?
cat gpurun_out/${T}_tgnn_window_kernel_stats.csv
cat gpurun_out/${T}_tgnn_bench.json
