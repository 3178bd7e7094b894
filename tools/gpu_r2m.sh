#!/bin/bash
# round 2: C3 A/B — DPP padding off (hazard checker clean) and 4 vs 5 waves/SIMD, at B = 65,536 and 8,192
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2m
mkdir -p $O
for L in default tools/abx/libmcpx_nopad.so tools/abx/libmcpx_w4.so tools/abx/libmcpx_w4nopad.so; do
  if [ $L = default ]; then E=""; else E="MCPX_LIB_PATH=$L"; fi
  env $E timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 4096 >> $O/ab.jsonl 2>> $O/ab.err || exit 3
done
