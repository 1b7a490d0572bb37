# fp16x3: plane swizzle (IKHIP_ANN_HSWZ) + SGPR wave / opaque LDS offset (uwl) in the
# working tree's libikhip.so against HEAD~'s build (libikhip_prev.so) and uwl alone;
# split epilogue (IKHIP_ANN_SPLIT_EPI 2 / 4 passes: s2, s4) on top.  ANN parity tests,
# bit identity, alternating bench lines, one SQ_LDS pass per build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k ann -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ann.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_ann.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for mode in fp16x3 fp32 bf16x6; do
  libs="libikhip_prev.so libikhip.so"
  if [ $mode = fp16x3 ]; then libs="$libs libikhip_s2.so libikhip_s4.so"; fi
  for lib in $libs; do
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/ann_bitcmp.py $mode > gpurun_out/annbit_${lib}_$mode.txt 2>&1 || exit $?
    echo "$mode $lib $(grep -v amdgpu.ids gpurun_out/annbit_${lib}_$mode.txt | awk '{print $NF}' | tr '\n' ' ')"
  done
done
MODE=fp16x3 bash tools/ann_ab.sh libikhip_prev.so libikhip_uwl.so libikhip.so libikhip_s2.so libikhip_s4.so libikhip_prev.so libikhip_uwl.so libikhip.so libikhip_s2.so libikhip_s4.so || exit $?
MODE=bf16x6 bash tools/ann_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so || exit $?
for lib in libikhip_prev.so libikhip.so libikhip_s2.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/lds_$lib -- python bench.py --method ann --ann-mode fp16x3 --steps 3 --warmup 1 --cpu-seconds 0 --secondary 0 --end-to-end 0 > gpurun_out/lds_$lib.log 2>&1 || exit $?
done
