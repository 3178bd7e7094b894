#!/bin/bash
# Register-resident workgroup LU iteration: its parity tests and the large-KKT bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-vr2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wg.py tests/test_fail_reason.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_wg.log 2>&1 || exit 3
Q=(--steps 3 --warmup 1 --cpu-sample 0 --host-runs 0)
timeout -k 10 300 python bench.py --n 128 --m 64 --global-batch 2048 --linear-solver reduced "${Q[@]}" > $O/bench_kkt256_reduced.json 2> $O/b1.err || exit 4
timeout -k 10 300 python bench.py --n 128 --m 64 --global-batch 2048 --linear-solver dense "${Q[@]}" > $O/bench_kkt256_dense.json 2> $O/b2.err || exit 5
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 > $O/bench_c4_t10.json 2> $O/b3.err || exit 6
