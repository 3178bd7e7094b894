#!/bin/bash
# quick GPU iteration: schur/reduced parity subset + benches + phase profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "golden or random_qp or edge or warm" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit 3
for ls in schur reduced; do timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --linear-solver $ls > gpurun_out/bench_${TAG}_$ls.json 2>> gpurun_out/bench_$TAG.err || exit 7; done
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --linear-solver schur > gpurun_out/bench_${TAG}_schur_generic.json 2>> gpurun_out/bench_$TAG.err || exit 5
for mode in schur schurgen; do timeout -k 10 120 ./tools/phase_profile 32 16 16384 $mode >> gpurun_out/phase_$TAG.txt 2>&1 || exit 6; done
