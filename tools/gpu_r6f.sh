#!/bin/bash
# 2-hop (comment-shaped, B = 600) same-box A/Bs: predictor waves, attention-backward load batches, predictor groups
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
T=${1:-r6f}
export BENCH_ARGS="--dataset tgbl-comment --batch 600 --layers 2 --window start"
bash tools/ab_bench.sh ${T}_libs default /root/repo/var/eb16/libtgnx.so /root/repo/var/pw8/libtgnx.so /root/repo/var/r4/libtgnx.so || exit 1
cat gpurun_out/${T}_libs_ab.txt
bash tools/ab_envs.sh ${T}_groups "-" "TGNX_PRED_GROUPS=600" "TGNX_PRED_GROUPS=150" || exit 1
cat gpurun_out/${T}_groups_ab.txt
