#!/bin/bash
# Round-2 evidence of the final build: GPU suite, smoke, then tools/gpu_profile.sh (bench line +
# rocprofv3 kernel trace of the same command + FETCH/WRITE/SQ/MFMA --pmc passes) for
#   c3      the driver's command (BASELINE C3, global 65,536 on 1 GPU)
#   c3b8192 the per-GPU shard of C3 at 8 GPUs (global 8,192 on 1 GPU)
#   c4      BASELINE C4 (lane change T=2, 1,024 games)
#   c5      BASELINE C5 (solve + rrule pullback, global 4,096)
# Summarise afterwards: python tools/prof_summary.py gpurun_out/prof_<name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > gpurun_out/ev/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev/smoke.log 2>&1 || exit 4
bash tools/gpu_profile.sh c3 || exit 5
bash tools/gpu_profile.sh c3b8192 --gpus 1 --global-batch 8192 --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 || exit 6
bash tools/gpu_profile.sh c4 --lane-change 2 --steps 5 --warmup 1 || exit 7
bash tools/gpu_profile.sh c5 --sens --steps 10 --warmup 2 || exit 8
