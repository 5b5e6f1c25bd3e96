#!/bin/bash
# HBM-side traffic per kernel launch from rocprofv3 PMC counters, collected as
# /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 PMC slots) prescribes: FETCH_SIZE and
# WRITE_SIZE in separate passes (they do not fit one TCC pass), no trace domains besides the
# kernel dispatches.  Writes gpurun_out/<tag>_pmc_{fetch,write}/ and gpurun_out/<tag>_pmc_traffic.json
# (merge into profiles/pmc_traffic.json with tools/pmc_summarize.py after the call; only gpurun_out/
# comes back from the box).
#   tools/pmc_traffic.sh <tag> [model]
tag=${1:-pmc}; model=${2:-tgn}
cd /tmp && export TMPDIR=/tmp
R=/root/repo
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -k 10 400 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/${tag}_pmc_$lc -o run -- \
    python3 $R/bench.py --model $model --only --steps 20 --warmup 5 --no-cpu-baseline --no-graph --probe-steps 1 \
    > $R/gpurun_out/${tag}_pmc_$lc.log 2>&1 || exit $?
done
python3 $R/tools/pmc_summarize.py $R/gpurun_out/${tag}_pmc_fetch $R/gpurun_out/${tag}_pmc_write \
  $R/gpurun_out/${tag}_pmc_traffic.json
