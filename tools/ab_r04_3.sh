set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "fabrik" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fabrik.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_fabrik.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in libikhip.so libikhip_unf.so libikhip_rprio.so libikhip_pcarry.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_$lib.txt 2>&1 || exit $?
  echo "$lib $(grep -v amdgpu.ids gpurun_out/bitcmp_$lib.txt | awk '{print $NF}' | tr '\n' ' ')"
done
bash tools/fab_ab.sh libikhip_unf.so libikhip.so libikhip_rprio.so libikhip_pcarry.so libikhip_unf.so libikhip.so libikhip_rprio.so libikhip_pcarry.so libikhip_unf.so libikhip.so libikhip_rprio.so libikhip_pcarry.so || exit $?
bash tools/ab_r04_4.sh || exit $?
