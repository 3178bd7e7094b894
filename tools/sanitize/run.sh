#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer builds (CPU only; GPU
# sanitizers are not available on the pool): the C oracle and the C ABI's host
# code (mcpx_api.cpp; device code untouched), each driven by its checks program.
#   tools/sanitize/run.sh [outdir]
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${1:-$ROOT/tools/sanitize/_build}
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g -O1"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:protect_shadow_gap=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
# 1. the oracle
gcc -std=c11 -ffp-contract=off $SAN -I"$ROOT/include" "$ROOT/oracle/ipm_oracle.c" \
    "$ROOT/tools/sanitize/oracle_checks.c" -o "$OUT/oracle_checks" -lm -lpthread
"$OUT/oracle_checks"
# 2. the C ABI host code, sanitized on the host side only, linked ahead of libmcpx.so
#    (whose kernels and launchers it calls)
/opt/rocm/bin/hipcc -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -Xarch_host -fsanitize=address \
    -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer -g -c "$ROOT/mcp_amd/csrc/mcpx_api.cpp" \
    -o "$OUT/mcpx_api_san.o"
/opt/rocm/lib/llvm/bin/clang++ -std=c++17 -fsanitize=address,undefined -g "$ROOT/tools/sanitize/abi_checks.cpp" \
    "$OUT/mcpx_api_san.o" -L"$ROOT/mcp_amd" -lmcpx -L/opt/rocm/lib -lamdhip64 \
    -Wl,-rpath,"$ROOT/mcp_amd" -Wl,-rpath,/opt/rocm/lib -lpthread -o "$OUT/abi_checks"
"$OUT/abi_checks"
