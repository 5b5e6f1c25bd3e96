#!/bin/bash
# kernel stats of the data-parallel compute floor (tools/dp_compute.py) at the given worlds -> gpurun_out/<tag>_dp<W>/
tag=$1; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for W in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_dp$W -o dp -- \
    python tools/dp_compute.py --worlds $W --steps 300 > gpurun_out/${tag}_dp$W.json 2> gpurun_out/${tag}_dp$W.err || exit $?
done
