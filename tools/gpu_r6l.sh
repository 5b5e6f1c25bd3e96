#!/bin/bash
# per-operator ops + the TGNN world-1 step with Adam folded into the gradient expansion: tests, then the
# same-box TGNN A/B (folded-Adam default vs the round-6 fold-only library and round 5) at B = 200 / 2000
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_module_ops.py tests/test_gpu_torch_ops.py tests/test_gpu_dropin.py tests/test_gpu_tgnn.py tests/test_gpu_tgnn_b2000.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
MODEL=tgnn bash tools/ab_bench.sh ${T}_b200 default /root/repo/var/r6fold/libtgnx.so /root/repo/var/r5/libtgnx.so || exit 1
cat gpurun_out/${T}_b200_ab.txt
MODEL=tgnn BENCH_ARGS="--batch 2000" bash tools/ab_bench.sh ${T}_b2000 default /root/repo/var/r6fold/libtgnx.so || exit 1
cat gpurun_out/${T}_b2000_ab.txt
