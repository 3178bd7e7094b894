#!/bin/bash
# Per-GPU work of the strong-scaling C3 run at N = 2, 4, 8 (global 65,536 sharded), on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/shard
mkdir -p $O
for G in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --gpus 1 --global-batch $G --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 > $O/bench_g$G.json 2> $O/bench_g$G.err || exit 3
done
timeout -k 10 300 python bench.py --sens --global-batch 512 --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_c5_g512.json 2> $O/bench_c5_g512.err || exit 4
timeout -k 10 300 python bench.py --lane-change 2 --global-batch 128 --steps 5 --warmup 1 --cpu-sample 0 > $O/bench_c4_g128.json 2> $O/bench_c4_g128.err || exit 5
