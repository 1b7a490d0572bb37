# fp16x3 next-layer prefetch (IKHIP_ANN_PREFETCH=1 build) against the default build:
# bit identity, then alternating bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in libikhip.so libikhip_pf.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py fp16x3 > gpurun_out/annbit_$lib.txt 2>&1 || exit $?
  echo "$lib $(grep -v amdgpu.ids gpurun_out/annbit_$lib.txt | awk '{print $NF}' | tr '\n' ' ')"
done
bash tools/ann_ab.sh libikhip.so libikhip_pf.so libikhip.so libikhip_pf.so || exit $?
