#!/bin/bash
# data-parallel compute floor A/B over runtime knobs: tools/gpu_dpab.sh <tag> "<ENV=..>" ... (2 rounds)
tag=$1; shift
cd "$(dirname "$0")/.."
out=gpurun_out/${tag}_dpab.txt; : > $out
for round in 1 2; do
  for e in "$@"; do
    r=$(env $e timeout -k 10 200 python tools/dp_compute.py --worlds 2 4 8 --steps 300 2>/dev/null) || exit 1
    echo "$e $(echo "$r" | python3 -c 'import json,sys; print([x["ms_per_step"] for x in json.loads(sys.stdin.read())["dp_compute_only"]])')" | tee -a $out
  done
done
