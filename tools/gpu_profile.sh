#!/bin/bash
# Evidence run: bench line, rocprofv3 kernel-trace stats of the same command,
# PMC passes (separately: FETCH_SIZE; WRITE_SIZE; SQ instruction counters), torchrun rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 2
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --cpu-sample 0 > $OUT/trace.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_write.log 2>&1 || exit 5
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --cpu-sample 0 > $OUT/pmc_sq.log 2>&1 || exit 6
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gather --steps 3 --cpu-sample 0 > $OUT/torchrun_gather.json 2> $OUT/torchrun.err || exit 7
