#!/bin/bash
# round 2: full GPU parity suite after the broadcast fix, the fixed x5 variant vs the oracle, C3/C4 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python tools/ab_c4/su5_check.py > $O/su5_check.jsonl 2> $O/su5_check.err || exit 4
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 > $O/bench_c3.json 2> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2>> $O/bench.err || exit 6
