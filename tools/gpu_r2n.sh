#!/bin/bash
# round 2: lone-wave vs loaded per-phase cycles of the C3 SCHUR kernel (s_memtime stamps, no DPP pads)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2n
mkdir -p $O
for B in 1024 4096 8192 65536; do timeout -k 10 120 ./tools/phase_profile 32 16 $B schur >> $O/phase.txt 2>&1 || exit 3; done
