#!/bin/bash
# Kernel A/B on the box: tools/ab_c3.py once per library (the product build first, then every
# tools/ablib/libmcpx_<name>.so named), same inputs, one JSON line per (library, batch).
#   tools/ab_libs.sh <out-file> "<ab_c3.py args>" name1 name2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 2
OUT=gpurun_out/${1:?out}; ARGS=$2; shift 2
mkdir -p "$(dirname "$OUT")"
timeout -k 10 240 python tools/ab_c3.py $ARGS >> "$OUT" 2>> "$OUT.err" || exit 3
for v in "$@"; do
  MCPX_LIB_PATH=tools/ablib/libmcpx_$v.so timeout -k 10 240 python tools/ab_c3.py $ARGS >> "$OUT" 2>> "$OUT.err" || exit 3
done
cat "$OUT"
