#!/bin/bash
# round 2: sparse nonlinear S formation — GPU suite, C4 phases, C4 T=2/T=10 bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 120 ./tools/nl_phase tools/abx/nl_t2_stamps.hsaco mcpx_nl_solve_schur tools/abx/theta_lane_t2_b1024.bin 40 50 10 1024 > $O/nl_phase.txt 2>&1 || exit 4
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4_t10.json 2>> $O/bench.err || exit 6
