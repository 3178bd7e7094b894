#!/bin/bash
# round 2: timeline of the host-buffer pipeline (kernel + memory-copy trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/trace -o run --output-format csv -- python3 tools/host_trace.py > $O/log.txt 2>&1 || exit 3
