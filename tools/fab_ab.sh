# A/B of FABRIK builds / knobs: bench lines at tol 1e-3 and 1e-5 for each
# argument LIB[:VAR=VAL[,VAR=VAL...]] (LIB under inversekinematicsann_amd/).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for spec in "$@"; do
  lib=${spec%%:*}
  envs=""
  if [ "$spec" != "$lib" ]; then envs=$(echo "${spec#*:}" | tr ',' ' '); fi
  tag=$(echo "$spec" | tr -c 'a-zA-Z0-9_.' '_')
  for tm in "1e-3 100" "1e-5 200"; do
    set -- $tm
    env $envs IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python bench.py --method fabrik --steps 30 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --tol $1 --max-iter $2 > gpurun_out/ab_${tag}_$1.json 2> gpurun_out/ab_${tag}_$1.err || exit $?
    echo "$spec tol=$1 $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d.get('kernels_ms', {}).items()})" gpurun_out/ab_${tag}_$1.json)"
  done
done
