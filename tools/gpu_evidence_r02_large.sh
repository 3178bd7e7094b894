#!/bin/bash
# Round-2 evidence of the large-KKT workgroup kernels on the final build, plus the nonlinear
# GPU parity file (C4 batch + edge inputs).  Summarise: python tools/prof_summary.py gpurun_out/prof_<name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev
timeout -k 10 600 python -u -m pytest tests/test_nonlinear.py -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/ev/pytest_nl.log 2>&1 || exit 3
bash tools/gpu_profile.sh c3n128 --n 128 --m 64 --linear-solver dense --global-batch 2048 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 4
bash tools/gpu_profile.sh c4t10 --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 || exit 5
