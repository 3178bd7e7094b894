#!/bin/bash
# Round-3 final evidence on the final tree: the GPU suite, smoke, the driver's bench line,
# then trace + PMC passes of the C3 / C5 / C2 / C4 bench lines and of the large-KKT lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final
mkdir -p $O
timeout -k 10 120 ./tools/nl_phase tools/ubench_data/nl_t2_stamps6.hsaco mcpx_nl_solve_schur tools/ubench_data/theta_lane_t2_b1024.bin 40 50 10 1024 64 6 > $O/phase_c4_6.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 5
bash tools/gpu_profile.sh c3 || exit 6
bash tools/gpu_profile.sh c5 --sens --steps 20 --warmup 5 || exit 7
bash tools/gpu_profile.sh c2 --n 16 --m 8 --global-batch 4096 --steps 20 --warmup 5 || exit 8
bash tools/gpu_profile.sh c4 --lane-change 2 --steps 10 --warmup 2 || exit 9
bash tools/gpu_profile.sh t10 --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 10
bash tools/gpu_profile.sh kkt256r --n 128 --m 64 --global-batch 2048 --linear-solver reduced --steps 3 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 11
