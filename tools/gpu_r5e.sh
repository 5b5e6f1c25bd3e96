#!/bin/bash
# round 5: stamps --top of var/st, then an A/B of the default build against var/e2
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TGNX_LIB=$PWD/var/st/libtgnx.so timeout -k 10 300 python tools/stamps.py --steps 20 --bins --top 6 > gpurun_out/${1}_stamps.txt 2>&1 || exit 1
STEPS=500 ROUNDS=2 tools/ab_r5.sh ${1} default $PWD/var/e2/libtgnx.so
