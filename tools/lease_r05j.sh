# r05 lease J: where the FABRIK iteration kernel's time goes after the lazy loop
# condition: the diagnostic build's per-wave breakdown at both tolerances, and the
# rocprof kernel trace of the FABRIK bench at each tolerance.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05j
timeout -k 10 300 python tools/fabrik_diag.py > gpurun_out/r05j/fabrik_diag.json 2> gpurun_out/r05j/fabrik_diag.err || exit $?
echo "diag ok"
for tm in "1e-3 100" "1e-5 200"; do
  set -- $tm
  rm -rf /tmp/r05j_trace
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05j_trace -o run -- python bench.py --method fabrik --steps 20 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --tol $1 --max-iter $2 > gpurun_out/r05j/bench_$1.json 2> gpurun_out/r05j/bench_$1.err || exit $?
  find /tmp/r05j_trace -name '*kernel_stats.csv' -exec cp {} gpurun_out/r05j/kernel_stats_$1.csv \;
  ls -la $(find /tmp/r05j_trace -type f) | awk '{print $5, $9}'
  echo "trace $1 ok"
done
