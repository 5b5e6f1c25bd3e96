#!/bin/bash
# PMC traffic (FETCH_SIZE, WRITE_SIZE passes) of the TGN bench step for one library: tools/pmc_variant.sh <tag> <lib>
tag=$1; lib=$2
R=/root/repo
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  sub=$(echo $ctr | cut -d_ -f1 | tr A-Z a-z)
  TGNX_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/${tag}_pmc/tgn_${sub} -o run -- \
    python3 $R/bench.py --model tgn --only --no-graph --steps 30 --warmup 5 --probe-steps 1 --no-cpu-baseline --no-train-loop --no-tcsr \
    > $R/gpurun_out/${tag}_pmc_tgn_${sub}.log 2>&1 || exit $?
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/${tag}_pmc > $R/gpurun_out/${tag}_pmc_traffic.json
