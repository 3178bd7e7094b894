#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2a
export TMPDIR=/tmp
(nproc; lscpu | head -20; python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)") > gpurun_out/r2a/env.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r2a/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench_default.json 2> gpurun_out/r2a/bench_default.err || exit 4
timeout -k 10 300 python bench.py --batch 8192 --steps 20 --warmup 5 --cpu-sample 0 > gpurun_out/r2a/bench_b8192.json 2>> gpurun_out/r2a/bench_default.err || exit 5
