#!/bin/bash
# Round-2 measurement: default bench line, the same command under rocprofv3 --kernel-trace --stats, and
# the other BASELINE configs on the TGN path.  Outputs under gpurun_out/ (copy the judged ones to profiles/).
set -o pipefail
R=/root/repo
T=${1:-m2}
cd $R
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- \
  python3 $R/bench.py > $R/gpurun_out/${T}_bench_under_rocprof.json 2> $R/gpurun_out/${T}_bench_under_rocprof.err || exit $?
cd $R
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-review --aggr mean --steps 300 --warmup 30 \
  --no-cpu-baseline --probe-steps 20 > gpurun_out/${T}_review.json 2> gpurun_out/${T}_review.err || exit $?
timeout -k 10 500 python bench.py --model tgn --only --dataset tgbl-coin --steps 300 --warmup 30 --no-cpu-baseline \
  --probe-steps 20 > gpurun_out/${T}_coin.json 2> gpurun_out/${T}_coin.err || exit $?
timeout -k 10 400 python bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 \
  --no-cpu-baseline --probe-steps 20 > gpurun_out/${T}_comment2.json 2> gpurun_out/${T}_comment2.err
cd $R && bash tools/pmc_traffic.sh ${T}
if [ -f $R/var/stamps/libtgnx.so ]; then
  TGNX_LIB=$R/var/stamps/libtgnx.so timeout -k 10 200 python tools/stamps.py --steps 20 --bins > gpurun_out/${T}_stamps.txt 2>&1
fi
