#!/bin/bash
# On the GPU box: SQ / SQC counters of the bench's eager TGN launches, one rocprofv3 pass per counter set.
#   tools/pmc_sq.sh <tag> "<counters set 1>" ["<counters set 2>" ...]  -> gpurun_out/<tag>_sq<i>/... + summary
tag=$1; shift
R=/root/repo
cd /tmp && export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/${tag}_sq$i -o run -- \
    python3 $R/bench.py --only --no-graph --steps 20 --warmup 5 --no-cpu-baseline --no-train-loop --no-tcsr \
    > $R/gpurun_out/${tag}_sq$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -3 $R/gpurun_out/${tag}_sq$i.log; exit 1; }
done
python3 $R/tools/pmc_kernels.py $R/gpurun_out/${tag}_sq* > $R/gpurun_out/${tag}_sq_summary.txt
cat $R/gpurun_out/${tag}_sq_summary.txt
