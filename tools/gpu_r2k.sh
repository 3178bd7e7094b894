#!/bin/bash
# round 2: generated-code register fix (fresh z loads, JIT CSE temps), division-free wg loops
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --lane-change 2 --steps 5 --warmup 1 > $O/bench_c4.json 2> $O/bench.err || exit 4
timeout -k 10 300 python bench.py --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4_t10.json 2>> $O/bench.err || exit 5
timeout -k 10 300 python bench.py --n 64 --m 32 --linear-solver dense --global-batch 8192 --steps 3 --warmup 1 --cpu-sample 0 --host-runs 0 > $O/bench_qp_n128.json 2>> $O/bench.err || exit 6
timeout -k 10 300 python bench.py --n 128 --m 64 --linear-solver dense --global-batch 2048 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 > $O/bench_qp_n256.json 2>> $O/bench.err || exit 7
