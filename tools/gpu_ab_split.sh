#!/bin/bash
# A/B: residual as two single-address-space streams (tools/abx/libmcpx_split.so) vs one flat stream

set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_split
mkdir -p $O
for L in default tools/abx/libmcpx_split.so default tools/abx/libmcpx_split.so; do
  if [ $L = default ]; then unset MCPX_LIB_PATH; else export MCPX_LIB_PATH=$L; fi
  timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 >> $O/ab.jsonl 2>> $O/ab.err || exit 3
done
unset MCPX_LIB_PATH
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_api.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 4
