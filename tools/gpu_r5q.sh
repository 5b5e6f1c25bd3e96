#!/bin/bash
# round 5 final: the other BASELINE configs on the TGN path (tools/measure_r5.sh B) and the DP compute floor
# (tools/gpu_dpfloor.sh), graph packet capture off as bench.py sets it -> gpurun_out/<tag>_*
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-q1}
bash tools/measure_r5.sh B $T || exit $?
bash tools/gpu_dpfloor.sh ${T}_dpf || exit $?
