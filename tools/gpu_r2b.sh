#!/bin/bash
# round 2: new bench line (strong-scaling default, host-API median, all-CPU baseline),
# the GPU bench tests, the C3 evidence run with the driver's exact command, counter list
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2b
mkdir -p $O
export TMPDIR=/tmp
rocprofv3 -L > $O/counters_list.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_bench.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_bench.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || exit 4
timeout -k 10 200 python bench.py --global-batch 8192 --steps 20 --warmup 5 --cpu-sample 0 --host-runs 0 > $O/bench_g8192.json 2>> $O/bench_default.err || exit 5
timeout -k 10 200 python bench.py --sens --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_c5.json 2>> $O/bench_default.err || exit 6
timeout -k 10 200 python bench.py --lane-change 2 --steps 5 --warmup 1 > $O/bench_c4.json 2>> $O/bench_default.err || exit 7
bash tools/gpu_profile.sh c3 --gpus 1 --steps 20 --warmup 5 || exit 8
