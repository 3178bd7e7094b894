#!/bin/bash
# round 2: sparse Schur formation of the nonlinear family (one-wave + workgroup), C4 T=2 / T=10 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_nonlinear.py tests/test_wg.py tests/test_bench.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench.err || exit 4
timeout -k 10 300 python bench.py --lane-change 2 --global-batch 8192 --steps 3 --warmup 1 --cpu-sample 0 > $O/bench_c4_b8192.json 2>> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4_t10.json 2>> $O/bench.err || exit 6
