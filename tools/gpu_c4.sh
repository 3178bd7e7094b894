#!/bin/bash
# BASELINE C4 evidence: lane-change bench line + rocprofv3 kernel-trace stats of the same command;
# then the default C3 bench line (picks up the refreshed PMC summary).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --lane-change 2 --batch 1024 --cpu-sample 256 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --lane-change 2 --batch 8192 --cpu-sample 0 > $OUT/bench_c4_b8192.json 2>> $OUT/bench_c4.err || exit 4
timeout -k 10 300 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 5
