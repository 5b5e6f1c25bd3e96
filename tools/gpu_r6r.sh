#!/bin/bash
# TGNN assemble at B = 2000: eight-keys-per-thread touch sort, register-sorted ring plan — phases, tests, A/B
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6r}
TGNX_LIB=/root/repo/var/timing/libtgnx.so timeout -k 10 200 python -u tools/phase_timing.py 2000 > gpurun_out/${T}_phase_b2000.txt 2>&1 || exit 1
cat gpurun_out/${T}_phase_b2000.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_tgnn.py tests/test_gpu_tgnn_b2000.py tests/test_gpu_sampler.py tests/test_gpu_torch_ops.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -60 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
MODEL=tgnn BENCH_ARGS="--batch 2000" bash tools/ab_bench.sh ${T}_b2000 default /root/repo/var/r6sort/libtgnx.so || exit 1
cat gpurun_out/${T}_b2000_ab.txt
MODEL=tgnn bash tools/ab_bench.sh ${T}_b200 default /root/repo/var/r6sort/libtgnx.so || exit 1
cat gpurun_out/${T}_b200_ab.txt
