#!/bin/bash
# Sanity run of the current build: GPU suite, smoke, the driver's bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sanity
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 4
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 5
