#!/bin/bash
# round 2: PCIe ceiling probe and host-path stream count A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/h2d_probe.py > $O/h2d_probe.jsonl 2> $O/h2d.err || exit 3
for S in 1 2 4 8; do
  MCPX_HOST_STREAMS=$S timeout -k 10 200 python bench.py --steps 2 --warmup 1 --cpu-sample 0 --host-runs 5 > $O/bench_host_s$S.json 2>> $O/bench.err || exit 4
done
