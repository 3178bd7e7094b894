#!/bin/bash
# first GPU contact: parity tests, a short bench, a rocprof kernel-trace summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/env.txt 2>&1
nproc >> gpurun_out/env.txt; lscpu | head -20 >> gpurun_out/env.txt
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
grep -q "passed" gpurun_out/pytest_gpu.log || exit 3
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 4
MCPX_GENERIC_KERNELS=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/bench1_generic.json 2>> gpurun_out/bench1.err || exit 5
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --n 16 --m 8 --batch 65536 --cpu-sample 2048 > gpurun_out/bench1_n32.json 2>> gpurun_out/bench1.err || exit 6
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof1.log 2>&1 || exit 7
