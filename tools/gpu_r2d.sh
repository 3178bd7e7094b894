#!/bin/bash
# round 2: workgroup-per-instance kernels vs the oracle, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wg.py -x -v -m gpu --timeout 240 --timeout-method thread > $O/pytest_wg.log 2>&1 || exit 3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 4
