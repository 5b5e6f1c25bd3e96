#!/bin/bash
# rocprofv3 kernel trace of the TGN bench with a library variant: tools/prof_variant.sh <tag> <lib>
tag=$1; lib=$2
cd /tmp && export TMPDIR=/tmp
export TGNX_LIB=$lib
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_prof -o run -- \
  python3 /root/repo/bench.py --model tgn --only --steps 100 --warmup 10 --no-cpu-baseline --no-graph --probe-steps 1 \
  > /root/repo/gpurun_out/${tag}_prof.log 2>&1
