#!/bin/bash
# 2-hop predictor reading its weights from L2: the 2-hop GPU tests, then the comment-shaped same-box A/B
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6h}
timeout -k 10 900 python -u -m pytest tests/test_gpu_tgn.py tests/test_gpu_tgn_configs.py tests/test_gpu_tgn_dp.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
BENCH_ARGS="--dataset tgbl-comment --batch 600 --layers 2 --window start" bash tools/ab_bench.sh ${T}_2hop default /root/repo/var/stage2/libtgnx.so /root/repo/var/r4/libtgnx.so || exit 1
cat gpurun_out/${T}_2hop_ab.txt
