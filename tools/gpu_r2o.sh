#!/bin/bash
# round 2: GPU suite on the reciprocal-GJ build, C3 A/B vs the previous build, C4 per-phase stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 4096 >> $O/ab.jsonl 2>> $O/ab.err || exit 4
MCPX_LIB_PATH=tools/abx/libmcpx_nopad.so timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 4096 >> $O/ab.jsonl 2>> $O/ab.err || exit 5
timeout -k 10 120 ./tools/nl_phase tools/abx/nl_t2_stamps.hsaco mcpx_nl_solve_schur tools/abx/theta_lane_t2_b1024.bin 40 50 10 1024 > $O/nl_phase.txt 2>&1 || exit 6
timeout -k 10 120 ./tools/nl_phase tools/abx/nl_t2_stamps.hsaco mcpx_nl_solve_schur tools/abx/theta_lane_t2_b1024.bin 40 50 10 64 >> $O/nl_phase.txt 2>&1 || exit 7
