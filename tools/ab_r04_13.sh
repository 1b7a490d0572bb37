# Split modes: the epilogue's activation before its barrier (IKHIP_ANN_ACT_EARLY=1, the
# working tree's libikhip.so) against after it (libikhip_prev.so, =0): ANN parity tests,
# bit identity, alternating bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k ann -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ann.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_ann.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for mode in fp16x3 bf16x6; do
  for lib in libikhip_prev.so libikhip.so; do
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py $mode > gpurun_out/annbit_${lib}_$mode.txt 2>&1 || exit $?
    echo "$mode $lib $(grep -v amdgpu.ids gpurun_out/annbit_${lib}_$mode.txt | awk '{print $NF}' | tr '\n' ' ')"
  done
done
MODE=fp16x3 bash tools/ann_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
MODE=bf16x6 bash tools/ann_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
