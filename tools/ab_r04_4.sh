set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libikhip.so libikhip_pf1.so libikhip_prevx.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py fp16x3 > gpurun_out/annbit_$lib.txt 2>&1 || exit $?
  echo "$lib $(grep -v amdgpu.ids gpurun_out/annbit_$lib.txt | awk '{print $NF}' | tr '\n' ' ')"
done
MODE=fp16x3 bash tools/ann_ab.sh libikhip.so libikhip_pf1.so libikhip_prevx.so libikhip.so libikhip_pf1.so libikhip_prevx.so || exit $?
