#!/bin/bash
# round 4, call 2: default bench line, DP compute-floor kernel stats at W = 2 / 8, stamps timeline (world 1)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/b2_bench.json 2> gpurun_out/b2_bench.err || exit $?
for W in 2 8; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/b2_dp$W -o dp -- python tools/dp_compute.py --worlds $W --steps 300 \
    > gpurun_out/b2_dp$W.json 2> gpurun_out/b2_dp$W.err || exit $?
done
TGNX_LIB=var/stamps/libtgnx.so timeout -k 10 240 python tools/stamps.py --bins > gpurun_out/b2_stamps.txt 2>&1
