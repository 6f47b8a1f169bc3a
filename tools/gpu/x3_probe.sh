# attribution of kfac_factor_tiles_x3's time on the MLP group: default build vs the
# timing probes (1 no DMA, 2 no split, 3 no MFMA), the shared-ring build, the fp32 kernel
set -o pipefail
mkdir -p gpurun_out/x3p
for R in 16384 32768; do
  for L in kfac_hip kfac_hip_p1 kfac_hip_p2 kfac_hip_p3 kfac_hip_x3s; do
    BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/lib$L.so timeout -k 10 120 python tools/x3_probe.py $R > gpurun_out/x3p/p_${L}_$R.log 2>&1 || { tail -20 gpurun_out/x3p/p_${L}_$R.log; exit 1; }
    grep rows= gpurun_out/x3p/p_${L}_$R.log
  done
  KFAC_TILES_X3=0 timeout -k 10 120 python tools/x3_probe.py $R > gpurun_out/x3p/p_f32_$R.log 2>&1 || exit 1
  grep rows= gpurun_out/x3p/p_f32_$R.log
done
