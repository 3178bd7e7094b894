#!/bin/bash
# GPU iteration loop: parity tests, then C3 bench (specialized + generic kernels).
# usage: bash tools/gpu_check.sh <tag> [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 4
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 "$@" > gpurun_out/bench_${TAG}_generic.json 2>> gpurun_out/bench_$TAG.err || exit 5
