#!/bin/bash
# Staged first runs of the band SCHUR kernel (diagnostic), least to most work; the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/band_stage.txt
S="timeout -k 5 60 python -u tools/band_stage.py"
$S 2 1 1 20 >> $O 2>&1 && $S 2 1 2 2 >> $O 2>&1 && $S 2 4 50 20 >> $O 2>&1 && $S 10 2 2 2 >> $O 2>&1 && $S 10 8 50 20 >> $O 2>&1 && $S 2 1024 50 20 >> $O 2>&1 && $S 10 256 50 20 >> $O 2>&1; echo "rc=$?" >> $O; cat $O
