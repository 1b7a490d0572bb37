# A/B of ANN library builds / knobs: one bench line per argument
# LIB[:VAR=VAL[,VAR=VAL...]] (LIB under inversekinematicsann_amd/) in mode $MODE.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MODE=${MODE:-fp16x3}
for spec in "$@"; do
  lib=${spec%%:*}
  envs=""
  if [ "$spec" != "$lib" ]; then envs=$(echo "${spec#*:}" | tr ',' ' '); fi
  tag=$(echo "$spec" | tr -c 'a-zA-Z0-9_.' '_')
  env $envs IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 300 python bench.py --method ann --ann-mode $MODE --steps ${STEPS:-10} --warmup 2 --cpu-seconds 0 --secondary 0 --end-to-end 0 > gpurun_out/annab_${tag}_$MODE.json 2> gpurun_out/annab_${tag}_$MODE.err || exit $?
  echo "$spec $MODE $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), round(d['value']/1e6,2), 'M/s frac', round(d['roofline']['frac'],3))" gpurun_out/annab_${tag}_$MODE.json)"
done
