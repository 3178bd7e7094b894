#!/bin/bash
# Ad-hoc GPU step without the prebuilt-module check (library-only changes; gpurun):
#   tools/gpu_quick.sh <out> "<pytest -k expr or empty>" [bench args ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/$1; K=$2; shift 2
mkdir -p "$O"
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 3; }
  tail -3 "$O/pytest.log"
fi
if [ $# -gt 0 ]; then
  timeout -k 10 600 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 4; }
  cut -c1-300 "$O/bench.json"
fi
