#!/bin/bash
# On the GPU box: the data-parallel compute floor (tools/dp_compute.py: rank 0 of a W-rank step on one device, exchange
# skipped) for BASELINE configs #4 (tgbl-coin, W 1 / 4 at global batch 800) and #5 (tgbl-comment 2-hop, W 1 / 8 at
# global batch 600), and the wiki headline's weak scaling (W 1 / 2 / 4 / 8 at 200 per rank) -> gpurun_out/<tag>_*.json
tag=${1:-dpf}
cd "$(dirname "$0")/.."
timeout -k 10 400 python tools/dp_compute.py --dataset tgbl-wiki --worlds 1 2 4 8 > gpurun_out/${tag}_wiki.json || exit $?
timeout -k 10 500 python tools/dp_compute.py --dataset tgbl-coin --worlds 1 4 --global-batch 800 --steps 100 > gpurun_out/${tag}_coin.json || exit $?
timeout -k 10 700 python tools/dp_compute.py --dataset tgbl-comment --layers 2 --worlds 1 8 --global-batch 600 --steps 100 > gpurun_out/${tag}_comment2.json || exit $?
