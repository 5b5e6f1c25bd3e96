#!/bin/bash
# round 5: rocprofv3 kernel stats of the comment-shaped 2-hop step, this build and the round-4 library
R=/root/repo
cd $R; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
for v in cur r4; do
  if [ $v = r4 ]; then export TGNX_LIB=$R/var/r4/libtgnx.so; else unset TGNX_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${1}_$v -o run -- \
    python3 $R/bench.py --model tgn --only --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --window start \
    --no-cpu-baseline --no-train-loop --no-tcsr --probe-steps 2 > $R/gpurun_out/${1}_$v.json 2>/dev/null || exit 1
done
