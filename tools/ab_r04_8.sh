set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in libikhip.so libikhip_spread.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 120 python tools/fab_bitcmp.py > gpurun_out/bitcmp_$lib.txt 2>&1 || exit $?
  echo "$lib $(grep -v amdgpu.ids gpurun_out/bitcmp_$lib.txt | awk '{print $NF}' | tr '\n' ' ')"
done
REPS=3 TOL=1e-3 MI=100 bash tools/fab_trace_ab.sh libikhip.so libikhip_spread.so || exit $?
mv gpurun_out/fabtrace gpurun_out/fabtrace_1e-3
REPS=2 TOL=1e-5 MI=200 bash tools/fab_trace_ab.sh libikhip.so libikhip_spread.so || exit $?
