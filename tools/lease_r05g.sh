# r05 lease G: the layered ANN GEMM with 2-D grouped tile order: parity, probe, counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/annb_pmc3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ann" > gpurun_out/pytest_ann.txt 2>&1; rc=$?
tail -2 gpurun_out/pytest_ann.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
for lib in libikhip.so libikhip_prev.so libikhip.so; do
  echo "== $lib"
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python tools/ann_big_probe.py 2>&1 | grep dims || exit 1
done
for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/annb_pmc3/$tag -- python tools/ann_big_probe.py 131072 4096x2 > gpurun_out/annb_pmc3/$tag.log 2>&1 || exit $?
done
echo done
