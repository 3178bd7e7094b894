#!/bin/bash
# The driver's round-end sequence on the final tree: GPU suite, smoke, default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 5
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 6
