#!/bin/bash
# Parity suite + C3 bench + kernel trace (iteration loop).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 3; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 4; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace_$TAG -o run --output-format csv -- python3 bench.py --cpu-sample 0 --steps 3 > gpurun_out/trace_$TAG.log 2>&1 || exit 5
head -5 gpurun_out/trace_$TAG/run_kernel_stats.csv
