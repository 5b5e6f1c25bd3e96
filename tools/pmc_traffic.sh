#!/bin/bash
# On the GPU box: HBM traffic per launch of the bench's probed kernels from PMC counters, one counter per
# rocprofv3 pass (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: they cannot share a pass), eager launches, over the
# bench's own TIMED window (--window mid: batches centred in the epoch; the prefill steps before it are in the
# trace too, so the summary keeps each kernel's dispatches of the timed steps only: config.timed_steps).
#   tools/pmc_traffic.sh <tag>  ->  gpurun_out/<tag>_pmc/{tgn,tgnn}_{fetch,write}/run_counter_collection.csv
#                                   and gpurun_out/<tag>_pmc_traffic.json (tools/pmc_summary.py)
tag=${1:-pmc}
R=/root/repo
cd /tmp && export TMPDIR=/tmp
for model in tgn tgnn; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    sub=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/${tag}_pmc/${model}_${sub} -o run -- \
      python3 $R/bench.py --model $model --only --no-graph --steps 30 --warmup 5 --window mid --no-probe --no-cpu-baseline --no-train-loop --no-tcsr \
      > $R/gpurun_out/${tag}_pmc_${model}_${sub}.json 2> $R/gpurun_out/${tag}_pmc_${model}_${sub}.log || exit $?
  done
done
win() { python3 -c 'import json,sys; a,b=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["config"]["timed_steps"]; print(f"{a}:{b}")' $1; }
PMC_WINDOW_TGN=$(win $R/gpurun_out/${tag}_pmc_tgn_fetch.json) PMC_WINDOW_TGNN=$(win $R/gpurun_out/${tag}_pmc_tgnn_fetch.json) \
  python3 $R/tools/pmc_summary.py $R/gpurun_out/${tag}_pmc > $R/gpurun_out/${tag}_pmc_traffic.json
