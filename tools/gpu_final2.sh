#!/bin/bash
# Round-end pass 2: the default bench command under rocprofv3 --kernel-trace --stats (+ the timed window's
# per-launch averages), then the PMC traffic passes over the timed window.  Usage: gpu_final2.sh TAG
set -o pipefail
T=${1:-r6f}
R=/root/repo
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd /tmp
timeout -k 10 700 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_bench_under_rocprof.err || exit $?
cd $R && python3 tools/rocprof_window.py gpurun_out/${T}_prof gpurun_out/${T}_bench_under_rocprof.json \
  > gpurun_out/${T}_window_kernel_stats.csv || exit $?
cat gpurun_out/${T}_window_kernel_stats.csv
bash tools/pmc_traffic.sh ${T} || exit $?
head -c 1500 gpurun_out/${T}_pmc_traffic.json
