#!/bin/bash
# Full evidence run: GPU parity suite, smoke, then tools/gpu_profile.sh (bench + rocprof trace + PMC + torchrun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 3; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 4; }
bash tools/gpu_profile.sh $TAG
