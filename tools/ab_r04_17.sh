# ANN fp32 tile shapes after the r04 register changes: MR = 1 (32-point tiles, two
# workgroups per CU: the default) against MR = 2 at 4 waves (IKHIP_ANN_MR=2) and MR = 2
# at 8 waves (libikhip_f8.so, IKHIP_ANN_FWAVES=8): bit identity, alternating bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "libikhip.so" "libikhip.so IKHIP_ANN_MR=2" "libikhip_f8.so IKHIP_ANN_MR=2"; do
  set -- $spec
  env ${2:-X_=1} IKHIP_LIB=$PWD/inversekinematicsann_amd/$1 timeout -k 10 120 python tools/ann_bitcmp.py fp32 > gpurun_out/annbit_tile.txt 2>&1 || exit $?
  echo "$spec $(grep -v amdgpu.ids gpurun_out/annbit_tile.txt | awk '{print $NF}' | tr '\n' ' ')"
done
MODE=fp32 bash tools/ann_ab.sh libikhip.so libikhip.so:IKHIP_ANN_MR=2 libikhip_f8.so:IKHIP_ANN_MR=2 libikhip.so libikhip.so:IKHIP_ANN_MR=2 libikhip_f8.so:IKHIP_ANN_MR=2 || exit $?
