#!/bin/bash
# TGNN edge-loop batching: parity tests, then same-box A/B of the variants at B = 200 and B = 2000
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6d}
timeout -k 10 600 python -u -m pytest tests/test_gpu_tgnn.py tests/test_gpu_tgnn_b2000.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
V="default /root/repo/var/r6c/libtgnx.so /root/repo/var/eb_ahead/libtgnx.so /root/repo/var/nb2/libtgnx.so /root/repo/var/bwd4/libtgnx.so /root/repo/var/ef8/libtgnx.so"
MODEL=tgnn bash tools/ab_bench.sh ${T}_b200 $V || exit 1
cat gpurun_out/${T}_b200_ab.txt
MODEL=tgnn BENCH_ARGS="--batch 2000" bash tools/ab_bench.sh ${T}_b2000 $V || exit 1
cat gpurun_out/${T}_b2000_ab.txt
