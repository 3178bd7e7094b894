#!/bin/bash
# round 2 (session 3): re-check HEAD on a fresh box — GPU suite, driver's C3 bench, C4 T=2/T=10
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench.err || exit 4
timeout -k 10 300 python bench.py --batch 8192 --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 > $O/bench_c3_b8192.json 2>> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 > $O/bench_c4.json 2>> $O/bench.err || exit 6
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4_t10.json 2>> $O/bench.err || exit 7
timeout -k 10 300 python bench.py --sens --steps 10 --warmup 2 > $O/bench_c5.json 2>> $O/bench.err || exit 8
