# r05 lease A: GPU tests, the default bench line, the 2-rank gloo rehearsal of the
# N > 1 bench (strong legs), the r03/r04 split-mode A/B.  Stops at a crash / limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/steps.txt
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread --maxfail=20
tail -3 gpurun_out/pytest_gpu.log
step bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5
tail -c 600 gpurun_out/bench_default.log; echo
step rehearsal_2rank 400 env IKHIP_DIST_BACKEND=gloo python bench.py --gpus 2 --gather 0 --steps 3 --warmup 1 --cpu-seconds 0 --end-to-end 0
python - <<'PY'
import json
d = json.loads(open("gpurun_out/rehearsal_2rank.log").read().strip().splitlines()[-1])
print("rehearsal", d["n_gpus"], d["config"].get("strong_legs"),
      {k: round(v["ms_per_step"], 3) for k, v in d.get("secondary", {}).items()})
PY
step ab_split 900 bash tools/ab_split_r05.sh
tail -4 gpurun_out/ab_split.log
