#!/bin/bash
# On the GPU box, one iteration: GPU tests (subset or all), stamps timeline (var/stamps), graph bench.
#   tools/gpu_iter.sh <tag> [pytest -k expr]
tag=${1:-it}; kexpr=${2:-}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
if [ -n "$kexpr" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$kexpr" > gpurun_out/${tag}_tests.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
fi
rc=$?; tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${tag}_tests.log | head -30; exit $rc; }
if [ -f var/stamps/libtgnx.so ]; then
  TGNX_LIB=$PWD/var/stamps/libtgnx.so timeout -k 10 200 python tools/stamps.py --steps 20 --bins > gpurun_out/${tag}_stamps.txt 2>&1 || exit $?
  sed -n '3,17p' gpurun_out/${tag}_stamps.txt
fi
timeout -k 10 300 python bench.py --model tgn --only --steps 500 --warmup 50 --no-cpu-baseline --probe-steps 20 > gpurun_out/${tag}_bench.json 2>gpurun_out/${tag}_bench.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print('bench', d['value'], d['ms_per_step'], {k: round(v,1) for k,v in d['kernels_us'].items()})"
