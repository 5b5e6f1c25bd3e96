#!/bin/bash
# On the GPU box: gpu tests, then the wiki (headline) and comment-shaped 2-hop bench lines -> gpurun_out/<tag>_*
tag=${1:-q}
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${tag}_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --only --no-cpu-baseline --probe-steps 20 --steps 300 > gpurun_out/${tag}_wiki.json 2> gpurun_out/${tag}_wiki.err || exit $?
timeout -k 10 400 python bench.py --only --no-cpu-baseline --dataset tgbl-comment --batch 600 --layers 2 --probe-steps 20 \
  --steps 100 --warmup 20 > gpurun_out/${tag}_comment2.json 2> gpurun_out/${tag}_comment2.err || exit $?
python3 - "$tag" <<'PY'
import json, sys
for f in ("wiki", "comment2"):
    d = json.load(open(f"gpurun_out/{sys.argv[1]}_{f}.json"))
    print(f, d["value"], d["ms_per_step"], {k: round(v, 1) for k, v in d["kernels_us"].items()})
PY
