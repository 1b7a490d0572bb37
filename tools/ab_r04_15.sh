# FABRIK retire step: the FK round trip from cos / sin taken from the angles' own geometry
# (IKHIP_FAB_FK_CS=1, working tree libikhip.so) against sincos of the angles (HEAD,
# libikhip_prev.so): FABRIK tests, bit identity of angles / iterations, rocprof windows.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "fabrik" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fab.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_fab.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for lib in libikhip_prev.so libikhip.so; do
  FAB_BITCMP_SPLIT=1 IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_$lib.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/bitcmp_$lib.txt | sed "s/^/$lib /"
done
REPS=3 TOL=1e-3 MI=100 bash tools/fab_trace_ab.sh libikhip_prev.so libikhip.so || exit $?
mv gpurun_out/fabtrace gpurun_out/fabtrace_1e-3
REPS=2 TOL=1e-5 MI=200 bash tools/fab_trace_ab.sh libikhip_prev.so libikhip.so || exit $?
