#!/bin/bash
# rocprofv3 kernel stats of the TGN path (eager) -> gpurun_out/<tag>_prof
tag=${1:-tgnp}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_prof -o run -- \
  python3 /root/repo/bench.py --model tgn --only --steps 100 --warmup 10 --no-cpu-baseline --no-graph --probe-steps 1 \
  > /root/repo/gpurun_out/${tag}_prof.log 2>&1 || exit $?
python3 - "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"/root/repo/gpurun_out/{sys.argv[1]}_prof/run_kernel_stats.csv")))
for r in rows[:40]:
    print(f"{r['Name'][:110]:110s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f}us")
PY
