#!/bin/bash
# A/B: default in-tree build vs an alternative build (MCPX_LIB_PATH), C3 bench x3 interleaved, alt parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
ALT=${2:?alt lib}
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/ab_${TAG}_def$i.json 2>/dev/null || exit 4
  MCPX_LIB_PATH=$ALT timeout -k 10 200 python bench.py --cpu-sample 0 > gpurun_out/ab_${TAG}_alt$i.json 2>/dev/null || exit 5
done
MCPX_LIB_PATH=$ALT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/ab_${TAG}_pytest.log; exit 6; }
tail -1 gpurun_out/ab_${TAG}_pytest.log
python - <<PY
import json
for v in ("def","alt"):
    r=[json.load(open(f"gpurun_out/ab_${TAG}_{v}{i}.json")) for i in (1,2,3)]
    print(v, ["%.3f"%(x["value"]/1e6) for x in r], ["%.3f"%x["roofline"]["kernel_ms"] for x in r])
PY
