cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab_kkt
for L in default tools/ablib/libmcpx_wgt1.so tools/ablib/libmcpx_wgt2.so tools/ablib/libmcpx_vrt1.so tools/ablib/libmcpx_vrt2.so; do
  if [ "$L" = default ]; then E=""; else E="MCPX_LIB_PATH=$L"; fi
  env $E timeout -k 10 200 python tools/ab_c3.py --n 128 --m 64 --solver reduced --batch 2048 --reps 3 >> gpurun_out/ab_kkt/ab.jsonl 2>>gpurun_out/ab_kkt/err.log || exit 3
done
cat gpurun_out/ab_kkt/ab.jsonl
