#!/bin/bash
# Evidence run for one bench configuration: the bench line, a rocprofv3 kernel trace
# of EXACTLY the same command, then separate --pmc passes (FETCH_SIZE; WRITE_SIZE;
# SQ instruction mix) of a 2-step run of the same configuration.
#   tools/gpu_profile.sh <out-name> [bench args...]     (default args: the driver's)
# Summarise afterwards with: python tools/prof_summary.py gpurun_out/prof_<out-name>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NAME=${1:-c3}; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--gpus 1 --steps 20 --warmup 5)
OUT=gpurun_out/prof_$NAME
mkdir -p $OUT
export TMPDIR=/tmp
echo "python3 bench.py ${ARGS[*]}" > $OUT/cmd.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > $OUT/bench.json 2> $OUT/trace.log || exit 3
P=(--steps 2 --warmup 0 --cpu-sample 0 --host-runs 0)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py "${ARGS[@]}" "${P[@]}" > $OUT/pmc_fetch.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py "${ARGS[@]}" "${P[@]}" > $OUT/pmc_write.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES -d $OUT/pmc_sq -o run --output-format csv -- python3 bench.py "${ARGS[@]}" "${P[@]}" > $OUT/pmc_sq.log 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o run --output-format csv -- python3 bench.py "${ARGS[@]}" "${P[@]}" > $OUT/pmc_mfma.log 2>&1 || exit 7
