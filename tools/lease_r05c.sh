# r05 lease C: where the fused quotient differs on real FABRIK inputs; the layered
# ANN path, HEAD's build against the working tree's, and its parity tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/quot_fab_check core_test_goals.f64 1e-3 100 || exit $?
timeout -k 10 120 tools/quot_fab_check core_test_goals.f64 1e-5 200 || exit $?
for lib in libikhip_prev.so libikhip.so; do
  echo "== $lib"
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python tools/ann_big_probe.py > gpurun_out/annbig_$lib.txt 2>&1 || { cat gpurun_out/annbig_$lib.txt; exit 1; }
  cat gpurun_out/annbig_$lib.txt
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "ann" > gpurun_out/pytest_ann.txt 2>&1; rc=$?
tail -3 gpurun_out/pytest_ann.txt; echo "pytest rc=$rc"
