# End-to-end (host arrays over PCIe) FABRIK time per 1M points for pipeline chunk
# sizes: one bench line per argument (IKHIP_PIPE_CHUNK points per chunk).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# an argument LIB:CHUNK runs inversekinematicsann_amd/LIB
for spec in "$@"; do
  c=${spec##*:}
  lib=libikhip.so
  if [ "$spec" != "$c" ]; then lib=${spec%%:*}; fi
  c=$(echo "$spec" | tr -c 'a-zA-Z0-9_.' '_')
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib IKHIP_PIPE_CHUNK=${spec##*:} timeout -k 10 300 python bench.py --method fabrik --steps 10 --warmup 2 --cpu-seconds 0 --secondary 0 --end-to-end 1 > gpurun_out/e2e_$c.json 2> gpurun_out/e2e_$c.err || exit $?
  echo "chunk $c $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=d['end_to_end']; print('device', round(d['ms_per_step'],3), 'pinned', round(e['ms_per_step'],3), 'pageable', round(e['pageable']['ms_per_step'],3))" gpurun_out/e2e_$c.json)"
done
