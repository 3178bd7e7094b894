#!/bin/bash
# GPU side of tools/band_debug.py: the early-exit variants in order, the first failure ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
O=gpurun_out/band_debug.txt
for N in 1 2 3 4 0; do
  timeout -k 5 40 python -u tools/band_debug.py run $N >> $O 2>&1 || { echo "variant $N: rc=$?" >> $O; cat $O; exit 3; }
done
cat $O
