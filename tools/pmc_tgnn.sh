#!/bin/bash
# On the GPU box: SQ / TCC counters of the TGNN train step's eager launches at a given batch (one rocprofv3 pass
# per counter set).  tools/pmc_tgnn.sh <tag> <batch> "<set 1>" ["<set 2>" ...] -> gpurun_out/<tag>_sq<i>/ + summary
tag=$1; B=$2; shift 2
R=/root/repo
cd /tmp && export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/${tag}_sq$i -o run -- \
    python3 $R/bench.py --model tgnn --only --no-graph --batch $B --steps 8 --warmup 3 --no-probe --no-cpu-baseline \
    --no-train-loop --no-tcsr --no-config1 > $R/gpurun_out/${tag}_sq$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -3 $R/gpurun_out/${tag}_sq$i.log; exit 1; }
done
python3 $R/tools/pmc_kernels.py $R/gpurun_out/${tag}_sq* > $R/gpurun_out/${tag}_sq_summary.txt
cat $R/gpurun_out/${tag}_sq_summary.txt
