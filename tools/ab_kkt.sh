# KKT-256 phase A/B (tools/ab_build.py variants with MCPX_WG_TWICE / MCPX_VR_TWICE): one
# ab_c3.py run per library, the product first.  tools/ab_kkt.sh <solver> <lib names...>
cd $GRAFT_REPO_ROOT
S=$1; shift
mkdir -p gpurun_out/ab_kkt
for L in default "$@"; do
  if [ "$L" = default ]; then E=""; else E="MCPX_LIB_PATH=tools/ablib/libmcpx_$L.so"; fi
  env $E timeout -k 10 200 python tools/ab_c3.py --n 128 --m 64 --solver $S --batch 2048 --reps 3 >> gpurun_out/ab_kkt/ab_$S.jsonl 2>>gpurun_out/ab_kkt/err.log || exit 3
done
cat gpurun_out/ab_kkt/ab_$S.jsonl
