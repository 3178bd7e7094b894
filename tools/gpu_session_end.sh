#!/bin/bash
# End-of-round check of the built tree (GPU suite, smoke, default bench) plus the C4
# back-substitution A/B (bs = product, bsd = DPP-broadcast variant).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/end
mkdir -p $O
MCPX_AB_OUT=tools/abv timeout -k 10 300 python tests/ab/ab_module.py run bs bsd --B 1024 > $O/ab_c4.txt 2>&1 || exit 2
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 5
