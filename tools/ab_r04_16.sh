# FABRIK queue tail in small grabs (IKHIP_FAB_TAIL points at the queue's end in grabs of
# IKHIP_FAB_TAIL_CHUNK; 0 = off): FABRIK tests with a tail on, bit identity, then
# rocprof timed windows over a small sweep, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
IKHIP_FAB_TAIL=131072 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "fabrik and not calc" -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fab.txt 2>&1
rc=$?; tail -2 gpurun_out/pytest_fab.txt; if [ $rc -ne 0 ]; then exit $rc; fi
for t in 0 131072; do
  IKHIP_FAB_TAIL=$t timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_tail$t.txt 2>&1 || exit $?
  echo "tail $t $(grep -v amdgpu.ids gpurun_out/bitcmp_tail$t.txt | awk '{print $NF}' | tr '\n' ' ')"
done
REPS=${REPS:-2} TOL=1e-3 MI=100 bash tools/fab_trace_ab.sh libikhip.so \
  libikhip.so:IKHIP_FAB_TAIL=32768,IKHIP_FAB_TAIL_CHUNK=8 \
  libikhip.so:IKHIP_FAB_TAIL=65536,IKHIP_FAB_TAIL_CHUNK=16 \
  libikhip.so:IKHIP_FAB_TAIL=131072,IKHIP_FAB_TAIL_CHUNK=16 \
  libikhip.so:IKHIP_FAB_TAIL=131072,IKHIP_FAB_TAIL_CHUNK=32 \
  libikhip.so:IKHIP_FAB_TAIL=262144,IKHIP_FAB_TAIL_CHUNK=32 2>&1 | grep build || exit $?
