# r06 lease B: FABRIK A/B (HEAD build vs working tree, rocprof, two interleaved
# pairs), then tools/lease_r06.sh (GPU tests, the profile round, fabrik_diag, the
# VALU split).  Stops at the first crash.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  bash tools/fab_ab_prof.sh gpurun_out/fabprof_$rep libikhip_prev.so libikhip.so || exit $?
done
bash tools/lease_r06.sh
