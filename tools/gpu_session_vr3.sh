#!/bin/bash
# Workgroup-kernel iteration: parity of the workgroup / nonlinear / sensitivity paths, the
# large-KKT bench lines with their FETCH/WRITE traffic, and the 5-phase C4 stamp profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-vr3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/nl_phase tools/ubench_data/nl_t2_stamps5.hsaco mcpx_nl_solve_schur tools/ubench_data/theta_lane_t2_b1024.bin 40 50 10 1024 64 5 > $O/phase_c4_5.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests/test_wg.py tests/test_fail_reason.py tests/test_nonlinear.py tests/test_sensitivity_nl.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_wg.log 2>&1 || exit 3
Q=(--steps 3 --warmup 1 --cpu-sample 0 --host-runs 0)
timeout -k 10 300 python bench.py --n 128 --m 64 --global-batch 2048 --linear-solver reduced "${Q[@]}" > $O/bench_kkt256_reduced.json 2> $O/b1.err || exit 4
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 > $O/bench_c4_t10.json 2> $O/b3.err || exit 6
P=(--steps 2 --warmup 0 --cpu-sample 0 --host-runs 0)
for cfg in "kkt256r --n 128 --m 64 --global-batch 2048 --linear-solver reduced" "t10 --lane-change 10 --global-batch 1024"; do
  set -- $cfg; name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$name -o run --output-format csv -- python3 bench.py "$@" "${P[@]}" > $O/pmc_fetch_$name.log 2>&1 || exit 7
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$name -o run --output-format csv -- python3 bench.py "$@" "${P[@]}" > $O/pmc_write_$name.log 2>&1 || exit 8
done
