#!/bin/bash
# round 2: look-ahead pivot search in the nonlinear LU — parity + C4 phases + bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_nonlinear.py tests/test_wg.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_nl.log 2>&1 || exit 3
timeout -k 10 120 ./tools/nl_phase tools/abx/nl_t2_stamps.hsaco mcpx_nl_solve_schur tools/abx/theta_lane_t2_b1024.bin 40 50 10 1024 > $O/nl_phase.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench.err || exit 5
