#!/bin/bash
# C4 A/B (lookahead LU, entry-parallel Schur formation), phase stamps, then the GPU suite + bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-s8}
mkdir -p $O
MCPX_AB_OUT=tools/abv timeout -k 10 300 python tests/ab/ab_module.py run product base la se --B 1024 > $O/ab_c4.txt 2>&1 || exit 2
timeout -k 10 120 ./tools/nl_phase tools/ubench_data/nl_t2_stamps.hsaco mcpx_nl_solve_schur tools/ubench_data/theta_lane_t2_b1024.bin 40 50 10 1024 > $O/phase_c4.txt 2>&1 || exit 3
timeout -k 10 300 python bench.py --lane-change 2 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err || exit 4
bash tools/gpu_check_r03.sh ${1:-s8} || exit 5
