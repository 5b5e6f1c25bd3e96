#!/bin/bash
# round-6 pass: full GPU suite, same-box A/Bs against the round-5 (and round-4) libraries, TGNN B=2000 profile
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
T=${1:-r6c}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_tests.log 2>&1 || { tail -40 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
bash tools/ab_bench.sh ${T} default /root/repo/var/r5/libtgnx.so || exit 1
cat gpurun_out/${T}_ab.txt
MODEL=tgnn bash tools/ab_bench.sh ${T}_tgnn default /root/repo/var/r5/libtgnx.so || exit 1
cat gpurun_out/${T}_tgnn_ab.txt
BENCH_ARGS="--dataset tgbl-comment --batch 600 --layers 2 --window start" bash tools/ab_bench.sh ${T}_2hop default /root/repo/var/r5/libtgnx.so /root/repo/var/r4/libtgnx.so || exit 1
cat gpurun_out/${T}_2hop_ab.txt
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${T}_prof_tgnn2000 -o run -- \
  python3 /root/repo/bench.py --model tgnn --only --batch 2000 --steps 20 --warmup 5 --no-cpu-baseline --no-probe \
  > /root/repo/gpurun_out/${T}_tgnn2000.json 2> /root/repo/gpurun_out/${T}_tgnn2000.err || exit 1
python3 /root/repo/tools/trace_stats.py $(find /root/repo/gpurun_out/${T}_prof_tgnn2000 -name "*kernel_trace.csv" | head -1) 16
