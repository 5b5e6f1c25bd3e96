#!/bin/bash
# Same-box A/B of library variants on one model / shape.  gpu_ab.sh TAG MODEL "BENCH_ARGS" lib1 [lib2 ...]
set -o pipefail
T=$1; M=$2; A=$3; shift 3
cd /root/repo && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MODEL=$M BENCH_ARGS="$A" bash tools/ab_bench.sh $T default "$@" || exit 1
cat gpurun_out/${T}_ab.txt
