# A/B of the v5 expand+depthwise timing variants (build_var/libast_hip_ed5_*.so, scripts/build_variants.sh)
# against the default library and v4 (AST_MB_ED5=0) on the config-5 k5 blocks.
set -e
O=gpurun_out/${TAG:-r06c}_ab5.txt; : > $O
for v in ${VARIANTS:-base v4 nost nodw noexp noA nohw}; do
  case $v in base) L=arbitrarystyletransfer_amd/libast_hip.so; E="";; v4) L=arbitrarystyletransfer_amd/libast_hip.so; E="AST_MB_ED5=0";; *) L=build_var/libast_hip_ed5_$v.so; E="";; esac
  echo "== $v" >> $O
  for c in ${CASES:-dec10 dec8}; do
    env $E AST_HIP_LIB=$L timeout -k 10 120 python scripts/bench_mb_blocks.py 32 $c 2>&1 | grep -v amdgpu.ids >> $O
  done
done
cat $O
