set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_profile.sh c3 || exit 3
bash tools/gpu_profile.sh c5 --sens --steps 20 --warmup 5 || exit 4
bash tools/gpu_profile.sh c2 --n 16 --m 8 --global-batch 4096 --steps 20 --warmup 5 || exit 5
bash tools/gpu_profile.sh c4 --lane-change 2 --steps 10 --warmup 2 || exit 6
