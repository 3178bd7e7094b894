#!/bin/bash
# The evidence of one bench line, in order (run through gpurun):
#   tools/evidence.sh <name> [bench args...]        (no args: the driver's command)
# 1. tools/gpu_profile.sh: the bench line, a rocprofv3 kernel trace of exactly that command and
#    separate --pmc passes of the same configuration;
# 2. tools/prof_summary.py: trace_/pmc_/kernel_stats_<key> summaries into gpurun_out/evidence/;
# 3. the bench line once more with MCPX_PROFILE_DIR=gpurun_out/evidence, so that its roofline
#    quotes those counters (bound from PMC, traffic, frac_trace): gpurun_out/evidence/bench_<key>.json.
# Copy gpurun_out/evidence/* into profiles/<round>/ afterwards (same build: bench.py keys them by
# lib hash and configuration).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
NAME=${1:?name}; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--gpus 1 --steps 20 --warmup 5)
DST=gpurun_out/evidence
mkdir -p $DST
export TMPDIR=/tmp
bash tools/gpu_profile.sh "$NAME" "${ARGS[@]}" || exit $?
python tools/prof_summary.py gpurun_out/prof_$NAME --dst $DST > gpurun_out/prof_$NAME/summary.log 2>&1 || { tail -5 gpurun_out/prof_$NAME/summary.log; exit 8; }
KEY=$(python -c "import json; print(json.loads(open('gpurun_out/prof_$NAME/bench.json').read().strip().splitlines()[-1])['evidence']['key'])") || exit 8
MCPX_PROFILE_DIR=$DST timeout -k 10 400 python bench.py "${ARGS[@]}" > $DST/bench_$KEY.json 2> gpurun_out/prof_$NAME/final.err || { tail -5 gpurun_out/prof_$NAME/final.err; exit 9; }
cut -c1-240 $DST/bench_$KEY.json
