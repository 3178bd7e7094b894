#!/bin/bash
# Guessed-pivot LU in the nonlinear SCHUR kernel: nonlinear GPU parity, then the C4 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4spec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_nonlinear.py tests/test_wg.py -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_nl.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --lane-change 2 --batch 8192 --steps 3 --warmup 1 --cpu-sample 0 > $O/bench_c4_b8192.json 2>> $O/bench.err || exit 6
