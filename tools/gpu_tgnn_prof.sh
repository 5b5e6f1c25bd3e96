#!/bin/bash
# TGNN kernel statistics (rocprofv3 --kernel-trace --stats) of the bench's TGNN line at a batch: gpu_tgnn_prof.sh TAG B
set -o pipefail
T=$1; B=$2
R=/root/repo
mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- \
  python3 $R/bench.py --model tgnn --only --no-cpu-baseline --no-train-loop --no-tcsr --no-config1 --no-probe --batch $B \
  --steps 100 --warmup 10 > $R/gpurun_out/${T}_bench.json 2> $R/gpurun_out/${T}_bench.err || exit $?
python3 - $R/gpurun_out/${T}_prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "tgnn" in r["Name"]:
        print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1000, 2))
PY
