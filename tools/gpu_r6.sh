#!/bin/bash
# round-6 GPU pass: selected tests (T=...), then a bench line.  Usage: gpurun -- bash tools/gpu_r6.sh TAG "TESTS" "BENCH_ARGS"
set -o pipefail
tag=${1:-r6}
tests=${2:-}
bargs=${3:-}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ -n "$tests" ]; then
  timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider $tests \
    > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
  tail -5 gpurun_out/${tag}_tests.log
fi
if [ "$bargs" != "none" ]; then
  timeout -k 10 600 python -u bench.py $bargs > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -30 gpurun_out/${tag}_bench.err; exit 1; }
  python - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c, r = d["config"], d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "edges", c.get("sampled_edges_per_step"), "probe_edges", c.get("probe_window_edges_per_step"))
print("roofline", r["kernel"], r["avg_launch_us"], r["frac"])
print("kernels", d["kernels_us"])
print("gpu_tgnn_config1", d.get("gpu_tgnn_config1"))
print("secondary", {k: d.get("secondary_path", {}).get(k) for k in ("value", "ms_per_step")})
PY
fi
