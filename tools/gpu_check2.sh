#!/bin/bash
# GPU parity (full -m gpu suite) then C3 / C2 benches; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python bench.py --cpu-sample 0 > gpurun_out/bench_${TAG}.json 2>> gpurun_out/bench_$TAG.err || exit 4
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --cpu-sample 0 --steps 3 > gpurun_out/bench_${TAG}_generic.json 2>> gpurun_out/bench_$TAG.err || exit 5
timeout -k 10 300 python bench.py --cpu-sample 0 --n 16 --m 8 --batch 65536 > gpurun_out/bench_${TAG}_c2.json 2>> gpurun_out/bench_$TAG.err || exit 6
if [ -x tools/phase_profile ]; then
  for mode in schur schurgen; do timeout -k 10 120 ./tools/phase_profile 32 16 16384 $mode >> gpurun_out/phase_$TAG.txt 2>&1 || exit 7; done
fi
