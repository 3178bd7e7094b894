#!/bin/bash
# round 2: rocprofv3 evidence of the workgroup-per-instance path (trace + PMC incl. MFMA counters)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash tools/gpu_profile.sh c4t10 --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 || exit 3
bash tools/gpu_profile.sh qpn256 --n 128 --m 64 --linear-solver dense --global-batch 2048 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 4
