#!/bin/bash
# round 2: reduced-system VJP — sensitivity parity on GPU + C5 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sensitivity.py tests/test_api.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --sens --steps 20 --warmup 5 --cpu-sample 0 > $O/bench_c5.json 2> $O/bench.err || exit 4
timeout -k 10 300 python bench.py --sens --batch 65536 --steps 10 --warmup 2 --cpu-sample 0 > $O/bench_c5_b65536.json 2>> $O/bench.err || exit 5
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_abi.py -x -q -m gpu --timeout 240 --timeout-method thread > $O/pytest_host.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-sample 0 > $O/bench_c3_host.json 2>> $O/bench.err || exit 7
