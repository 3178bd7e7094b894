#!/bin/bash
# Register-resident workgroup LU (lu_vr.hpp): the GPU suite, then the large-KKT bench lines
# (KKT 256 REDUCED = VR, KKT 256 DENSE = HBM LU, lane change T = 10 SCHUR = VR) with
# traces and FETCH/WRITE passes, and the 5-phase C4 stamp profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-vr}
mkdir -p $O
timeout -k 10 120 ./tools/nl_phase tools/ubench_data/nl_t2_stamps5.hsaco mcpx_nl_solve_schur tools/ubench_data/theta_lane_t2_b1024.bin 40 50 10 1024 64 5 > $O/phase_c4_5.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
Q=(--steps 3 --warmup 1 --cpu-sample 0 --host-runs 0)
timeout -k 10 300 python bench.py --n 128 --m 64 --global-batch 2048 --linear-solver reduced "${Q[@]}" > $O/bench_kkt256_reduced.json 2> $O/b1.err || exit 4
timeout -k 10 300 python bench.py --n 128 --m 64 --global-batch 2048 --linear-solver dense "${Q[@]}" > $O/bench_kkt256_dense.json 2> $O/b2.err || exit 5
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 > $O/bench_c4_t10.json 2> $O/b3.err || exit 6
bash tools/gpu_profile.sh kkt256r --n 128 --m 64 --global-batch 2048 --linear-solver reduced "${Q[@]}" || exit 7
bash tools/gpu_profile.sh t10 --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 8
