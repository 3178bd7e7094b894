#!/bin/bash
# C4 A/B: 2-D back substitution (bs) against the product module, with 5-phase stamps of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-bs}
mkdir -p $O
MCPX_AB_OUT=tools/abv timeout -k 10 300 python tests/ab/ab_module.py run product se bs --B 1024 > $O/ab_c4.txt 2>&1 || exit 2
timeout -k 10 120 ./tools/nl_phase tools/ubench_data/nl_t2_stamps5_bs.hsaco mcpx_nl_solve_schur tools/ubench_data/theta_lane_t2_b1024.bin 40 50 10 1024 64 5 > $O/phase_c4_5_bs.txt 2>&1 || exit 3
