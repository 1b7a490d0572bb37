set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libikhip.so libikhip_rprio.so libikhip_pcarry.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_$lib.txt 2>&1 || exit $?
done
cat gpurun_out/bitcmp_*.txt
bash tools/fab_ab.sh libikhip.so libikhip_rprio.so libikhip_pcarry.so libikhip.so libikhip_rprio.so libikhip_pcarry.so || exit $?
bash tools/ann_traffic_ab.sh || exit $?
