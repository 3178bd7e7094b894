#!/bin/bash
# bench-only GPU iteration: C3 with every linear solver + phase profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
mkdir -p gpurun_out
for ls in reduced schur dense; do timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --linear-solver $ls > gpurun_out/bench_${TAG}_$ls.json 2>> gpurun_out/bench_$TAG.err || exit 7; done
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 --linear-solver schur > gpurun_out/bench_${TAG}_schur_generic.json 2>> gpurun_out/bench_$TAG.err || exit 5
for mode in spec schur schurgen; do timeout -k 10 120 ./tools/phase_profile 32 16 16384 $mode >> gpurun_out/phase_$TAG.txt 2>&1 || exit 6; done
