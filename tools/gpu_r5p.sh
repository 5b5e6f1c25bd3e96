#!/bin/bash
# round 5, graph packet capture off (bench.py / tgnx set DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): full GPU suite under it,
# then the default bench line and the same command under rocprofv3 --kernel-trace --stats -> gpurun_out/<tag>_*
set -o pipefail
R=/root/repo
T=${1:-p1}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_bench_under_rocprof.err || exit $?
