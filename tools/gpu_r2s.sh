#!/bin/bash
# round 2: C3 A/B — GJ pivots recorded by v_writelane (no per-lane selects, no SGPR spills)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2s
mkdir -p $O
timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 4096 >> $O/ab.jsonl 2>> $O/ab.err || exit 3
MCPX_LIB_PATH=tools/abx/libmcpx_wl.so timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 4096 >> $O/ab.jsonl 2>> $O/ab.err || exit 4
timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 >> $O/ab.jsonl 2>> $O/ab.err || exit 5
MCPX_LIB_PATH=tools/abx/libmcpx_wl.so timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 >> $O/ab.jsonl 2>> $O/ab.err || exit 6
