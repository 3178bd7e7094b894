#!/bin/bash
# round 2: host-buffer pipeline (one upload stream, cached streams): GPU suite, variants, trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 3
timeout -k 10 400 python tools/host_ab.py > $O/host_ab3.jsonl 2>> $O/err.log || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace3 -o run --output-format csv -- python3 tools/host_trace.py > $O/log3.txt 2>&1 || exit 5
