#!/bin/bash
# A/B: uniform fast reciprocal in the Gauss-Jordan (product build) vs the compiler's
# division (tools/abx/libmcpx_ldsa.so); QP parity tests; C4 wave vs workgroup probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_rcp
mkdir -p $O
for L in default tools/abx/libmcpx_ldsa.so default tools/abx/libmcpx_ldsa.so; do
  if [ $L = default ]; then unset MCPX_LIB_PATH; else export MCPX_LIB_PATH=$L; fi
  timeout -k 10 200 python tools/ab_c3.py --batch 65536 8192 >> $O/ab.jsonl 2>> $O/ab.err || exit 3
done
unset MCPX_LIB_PATH
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_api.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 4
timeout -k 10 300 python tools/c4_wg_probe.py 2 > $O/c4_wg_probe.txt 2>&1 || exit 5
