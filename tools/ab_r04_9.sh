set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "ann_vs_oracle or layered or width_cap or bad_models" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_big.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_big.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in libikhip_a2.so libikhip_sw.so; do
  echo "== $lib"
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python tools/ann_big_probe.py 262144 2>&1 | grep -v amdgpu || exit $?
done
