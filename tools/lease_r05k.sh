# r05 lease K: the refill threshold re-swept after the lazy loop condition
# (IKHIP_FAB_REFILL 6 / 8 / 12 / 16, same box), and the rocprof kernel trace of
# the FABRIK bench at both tolerances (csv stats only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05k
timeout -k 10 1000 bash tools/fab_ab.sh libikhip.so libikhip_rf16.so libikhip_rf20.so libikhip_rf24.so libikhip_rf32.so libikhip.so libikhip_rf16.so libikhip_rf20.so libikhip_rf24.so libikhip_rf32.so || exit $?
exit 0
for tm in "1e-3 100" "1e-5 200"; do
  set -- $tm
  rm -rf /tmp/r05k_trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05k_trace -o run -- python bench.py --method fabrik --steps 20 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --tol $1 --max-iter $2 > gpurun_out/r05k/bench_$1.json 2> gpurun_out/r05k/bench_$1.err || exit $?
  find /tmp/r05k_trace -name '*kernel_stats.csv' -exec cp {} gpurun_out/r05k/kernel_stats_$1.csv \;
  echo "trace $1 ok"
done
