#!/bin/bash
# Round-3 end check on the final tree: GPU suite, smoke, the driver's bench line, and the
# C3 trace + PMC passes of that command (profiles keyed to this build's lib hash).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 5
bash tools/gpu_profile.sh c3 || exit 6
