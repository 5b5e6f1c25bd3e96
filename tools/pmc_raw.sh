#!/bin/bash
# Raw memory-side request counters (read: 128/64/32-B requests, write: all / 64-B) of the TGN bench step, one
# TCC group per pass: tools/pmc_raw.sh <tag> [lib]  -> gpurun_out/<tag>_pmc/tgn_{rd,wr}/, summarised with the
# FETCH_SIZE / WRITE_SIZE passes of the same tag (tools/pmc_variant.sh) by tools/pmc_summary.py
tag=$1; lib=${2:-/root/repo/tgb-tgn-dgl_amd/tgnx/libtgnx.so}
R=/root/repo
cd /tmp && export TMPDIR=/tmp
run() {  # sub counters
  local sub=$1; shift
  TGNX_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/${tag}_pmc/tgn_${sub} -o run -- \
    python3 $R/bench.py --model tgn --only --no-graph --steps 30 --warmup 5 --window mid --no-probe --no-cpu-baseline --no-train-loop --no-tcsr \
    > $R/gpurun_out/${tag}_pmc_tgn_${sub}.log 2>&1
}
run rd TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum || exit $?
run wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum || exit $?
python3 $R/tools/pmc_summary.py $R/gpurun_out/${tag}_pmc > $R/gpurun_out/${tag}_pmc_traffic.json
