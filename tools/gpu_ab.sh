#!/bin/bash
# A/B of two library builds on the C3 bench + GPU parity of the default build + phase profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
ALT=${2:-tools/exp/libmcpx_rfl.so}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_${TAG}_default.json 2>> gpurun_out/bench_$TAG.err || exit 4
MCPX_LIB_PATH=$ALT timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_${TAG}_alt.json 2>> gpurun_out/bench_$TAG.err || exit 5
timeout -k 10 300 python bench.py --cpu-sample 0 --n 16 --m 8 --batch 65536 > gpurun_out/bench_${TAG}_c2big.json 2>> gpurun_out/bench_$TAG.err || exit 6
for mode in schur schurgen; do timeout -k 10 120 ./tools/phase_profile 32 16 16384 $mode >> gpurun_out/phase_$TAG.txt 2>&1 || exit 7; done
