#!/bin/bash
# split-K last-arriver (TGNX_SPLITK_LA): the TGN GPU tests, then the wiki same-box A/B against the fixup form
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6j}
timeout -k 10 900 python -u -m pytest tests/test_gpu_tgn.py tests/test_gpu_tgn_epochs.py tests/test_gpu_pyg_dropin.py tests/test_gpu_tgn_rccl.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
bash tools/ab_bench.sh ${T}_wiki default /root/repo/var/nola/libtgnx.so || exit 1
cat gpurun_out/${T}_wiki_ab.txt
