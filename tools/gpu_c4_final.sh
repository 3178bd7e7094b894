#!/bin/bash
# GPU parity suite + smoke + BASELINE C4 bench line and its rocprofv3 kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c4f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 3; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 4; }
timeout -k 10 300 python bench.py --lane-change 2 --batch 1024 --cpu-sample 1024 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 6
timeout -k 10 300 python bench.py --lane-change 2 --batch 8192 --cpu-sample 0 > $OUT/bench_c4_b8192.json 2>> $OUT/bench_c4.err || exit 7
