#!/bin/bash
# On the GPU box: HBM traffic per launch of the bench's probed kernels from PMC counters, one counter per
# rocprofv3 pass (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: they cannot share a pass), eager launches.
#   tools/pmc_traffic.sh <tag>  ->  gpurun_out/<tag>_pmc/{tgn,tgnn}_{fetch,write}/run_counter_collection.csv
#                                   and gpurun_out/<tag>_pmc_traffic.json (tools/pmc_summary.py)
tag=${1:-pmc}
R=/root/repo
cd /tmp && export TMPDIR=/tmp
for model in tgn tgnn; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    sub=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/${tag}_pmc/${model}_${sub} -o run -- \
      python3 $R/bench.py --model $model --only --no-graph --steps 30 --warmup 5 --probe-steps 1 --window start --no-cpu-baseline --no-train-loop --no-tcsr \
      > $R/gpurun_out/${tag}_pmc_${model}_${sub}.log 2>&1 || exit $?
  done
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/${tag}_pmc > $R/gpurun_out/${tag}_pmc_traffic.json
