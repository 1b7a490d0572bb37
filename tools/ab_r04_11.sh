# ANN register-pressure knobs: SGPR wave index + per-layer opaque LDS offset (uwl, l),
# and the fp16x3 next-layer prefetch on top (pf, pfl late, pfb with bias); bit
# identity first, then alternating bench lines per mode.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mode in fp16x3 fp32 bf16x6; do
  for lib in libikhip.so libikhip_uwl.so libikhip_pf.so; do
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py $mode > gpurun_out/annbit_${lib}_$mode.txt 2>&1 || exit $?
    echo "$mode $lib $(grep -v amdgpu.ids gpurun_out/annbit_${lib}_$mode.txt | awk '{print $NF}' | tr '\n' ' ')"
  done
done
MODE=fp16x3 bash tools/ann_ab.sh libikhip.so libikhip_uwl.so libikhip_l.so libikhip_pf.so libikhip_pfl.so libikhip_pfb.so libikhip.so libikhip_uwl.so libikhip_pf.so libikhip_pfl.so || exit $?
MODE=fp32 bash tools/ann_ab.sh libikhip.so libikhip_uwl.so libikhip.so libikhip_uwl.so || exit $?
MODE=bf16x6 bash tools/ann_ab.sh libikhip.so libikhip_uwl.so libikhip.so libikhip_uwl.so || exit $?
