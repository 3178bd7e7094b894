#!/bin/bash
# Everything round 2 commits as evidence, on the final build, in one call:
# GPU suite + smoke, the BASELINE lines with traces and PMC passes (tools/gpu_profile.sh),
# the large-KKT lines, and the per-GPU shard sizes of the strong-scaling configs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_evidence_r02.sh || exit $?
bash tools/gpu_profile.sh c3n128 --n 128 --m 64 --linear-solver dense --global-batch 2048 --steps 2 --warmup 1 --cpu-sample 0 --host-runs 0 || exit 10
bash tools/gpu_profile.sh c4t10 --lane-change 10 --global-batch 1024 --steps 2 --warmup 1 --cpu-sample 0 || exit 11
bash tools/gpu_shard_proxy.sh || exit 12
timeout -k 10 300 python bench.py --lane-change 2 --batch 8192 --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/ev/bench_c4_b8192.json 2> gpurun_out/ev/bench_c4_b8192.err || exit 13
