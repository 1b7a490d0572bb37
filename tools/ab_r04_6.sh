set -o pipefail
cd $GRAFT_REPO_ROOT
REPS=3 TOL=1e-3 MI=100 bash tools/fab_trace_ab.sh libikhip_unf_noprio.so libikhip.so || exit $?
mv gpurun_out/fabtrace gpurun_out/fabtrace_1e-3
REPS=2 TOL=1e-5 MI=200 bash tools/fab_trace_ab.sh libikhip_unf_noprio.so libikhip.so || exit $?
