#!/bin/bash
# rocprofv3 kernel stats of the comment-shaped 2-hop bench: pipelined step vs parity-set step with its node-set walk
# as its own launch (TGNX_WALK_AT=2) -> gpurun_out/<tag>_{pipe,pp}/
tag=${1:-cp}
R=/root/repo
cd /tmp && export TMPDIR=/tmp
A="--model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 5"
TGNX_PP_2HOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_pipe -o run -- \
  python3 $R/bench.py $A > $R/gpurun_out/${tag}_pipe.json 2> $R/gpurun_out/${tag}_pipe.err || exit $?
TGNX_PP_2HOP=1 TGNX_WALK_AT=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_pp -o run -- \
  python3 $R/bench.py $A > $R/gpurun_out/${tag}_pp.json 2> $R/gpurun_out/${tag}_pp.err || exit $?
