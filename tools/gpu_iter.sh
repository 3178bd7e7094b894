#!/bin/bash
# one GPU iteration: parity tests + C3 bench (spec & generic) + phase profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 4
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench_${TAG}_generic.json 2>> gpurun_out/bench_$TAG.err || exit 5
for ls in schur dense; do timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --linear-solver $ls > gpurun_out/bench_${TAG}_$ls.json 2>> gpurun_out/bench_$TAG.err || exit 7; done
for mode in spec schur schurgen; do timeout -k 10 120 ./tools/phase_profile 32 16 16384 $mode >> gpurun_out/phase_$TAG.txt 2>&1 || exit 6; done
