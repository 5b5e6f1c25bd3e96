#!/bin/bash
# round 5 final check: smoke(), then tools/gpu_r5p.sh (full GPU suite, default bench, bench under rocprofv3)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${1:-f1}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
bash tools/gpu_r5p.sh $T
