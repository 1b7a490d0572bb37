# FABRIK A/B with per-kernel times: each LIB (under inversekinematicsann_amd/) runs the
# FABRIK-only bench under rocprofv3 --kernel-trace, REPS times interleaved, at TOL / MI;
# tools/fab_trace_summary.py prints each run's step and the timed window's kernel averages.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fabtrace
mkdir -p $OUT
REPS=${REPS:-3}
TOL=${TOL:-1e-3}
MI=${MI:-100}
for r in $(seq 1 $REPS); do
  for spec in "$@"; do  # LIB[:VAR=VAL[,VAR=VAL...]]
    lib=${spec%%:*}
    envs=""
    if [ "$spec" != "$lib" ]; then envs=$(echo "${spec#*:}" | tr ',' ' '); fi
    tag=$(echo "${spec%.so*}${spec#*.so}" | tr -c 'a-zA-Z0-9_\n' '_')_${TOL}_$r
    env $envs IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -s KILL 120 rocprofv3 --kernel-trace \
        --output-format csv -d $OUT/$tag -- python bench.py --method fabrik --tol $TOL \
        --max-iter $MI --secondary 0 --cpu-seconds 0 --end-to-end 0 --cold 0 --steps 30 \
        --warmup 5 > $OUT/$tag.json 2> $OUT/$tag.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; exit $rc; fi
  done
done
python tools/fab_trace_summary.py --dir $OUT --steps 30
