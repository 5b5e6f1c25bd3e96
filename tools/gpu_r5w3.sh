#!/bin/bash
# round 5: the dW_cell launch's waves-per-SIMD floor (TGNX_W3_WAVES 7, the default build, against 0 =
# the compiler's register count, var/w3w0) at the wiki B = 200 step, TGN.yml's B = 2,000 and the comment-shaped
# 2-hop B = 600 step -> gpurun_out/<tag>_{wiki,b2000,c2}_ab.txt
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-w3}
W0=/root/repo/var/w3w0/libtgnx.so
STEPS=300 ROUNDS=2 tools/ab_r5.sh ${T}_wiki default $W0 || exit 1
STEPS=40 ROUNDS=2 BENCH_ARGS="--batch 2000 --window start --warmup 10" tools/ab_r5.sh ${T}_b2000 default $W0 || exit 1
STEPS=60 ROUNDS=2 BENCH_ARGS="--dataset tgbl-comment --batch 600 --layers 2 --window start" tools/ab_r5.sh ${T}_c2 default $W0 || exit 1
