set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libikhip.so libikhip_claim1.so; do
  for m in fp32 fp16x3; do
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py $m > gpurun_out/annbit_${lib}_$m.txt 2>&1 || exit $?
  done
done
IKHIP_LIB=$PWD/inversekinematicsann_amd/libikhip_rp_pc.so timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_rp_pc.txt 2>&1 || exit $?
grep -h "" gpurun_out/annbit_*.txt gpurun_out/bitcmp_rp_pc.txt | grep -v amdgpu.ids
MODE=fp32 bash tools/ann_ab.sh libikhip.so libikhip_claim1.so libikhip.so libikhip_claim1.so || exit $?
MODE=fp16x3 bash tools/ann_ab.sh libikhip.so libikhip_claim1.so libikhip.so libikhip_claim1.so || exit $?
LIBS="libikhip.so libikhip_claim1.so" bash tools/ann_traffic_ab.sh || exit $?
bash tools/fab_ab.sh libikhip.so libikhip_rp_pc.so libikhip.so libikhip_rp_pc.so || exit $?
