#!/bin/bash
# On the GPU box: gpu tests, graph bench, eager rocprof kernel stats -> gpurun_out/<tag>_*
tag=${1:-chk}
cd "$(dirname "$0")/.."
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
timeout -k 10 240 python bench.py --steps 300 --warmup 30 --no-cpu-baseline > gpurun_out/${tag}_bench.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' gpurun_out/${tag}_bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${tag}_prof -o run -- \
  python3 /root/repo/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-graph > /root/repo/gpurun_out/${tag}_prof.log 2>&1 || exit $?
python3 - "$tag" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"/root/repo/gpurun_out/{sys.argv[1]}_prof/run_kernel_stats.csv")))
steps = max(int(r["Calls"]) for r in rows if "tgnn_assemble" in r["Name"])
tot = 0
for r in rows:
    c = int(r["Calls"]); a = float(r["AverageNs"]) / 1e3
    if c >= 400:
        tot += a * c / steps
        print(f"{r['Name'][:50]:50s} {c:6d} {a:8.2f}us")
print("per-step kernel sum %.1f us" % tot)
PY
