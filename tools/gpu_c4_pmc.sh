#!/bin/bash
# PMC passes (FETCH_SIZE; WRITE_SIZE) of the BASELINE C4 bench command, one counter group per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_c4
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_write.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --lane-change 2 --batch 1024 --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_sq.log 2>&1 || exit 5
