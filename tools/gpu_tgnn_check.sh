#!/bin/bash
# TGNN change check: the TGNN GPU tests, then the same-box TGNN A/B at B = 200 and 2,000 against a baseline library.
#   gpu_tgnn_check.sh TAG BASELINE_LIB
set -o pipefail
T=$1; BASE=$2
cd /root/repo && mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_tgnn.py tests/test_gpu_tgnn_b2000.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -50 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
bash tools/gpu_ab.sh ${T}_b200 tgnn "" $BASE || exit 1
bash tools/gpu_ab.sh ${T}_b2000 tgnn "--batch 2000" $BASE || exit 1
