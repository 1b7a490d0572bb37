cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/spread
for w in 2 5 2 5 2 5; do
  for tol in 1e-3; do
    timeout -k 10 120 python bench.py --method fabrik --secondary 0 --cpu-seconds 0 --end-to-end 0 --cold 0 --steps 20 --warmup $w > gpurun_out/spread/w${w}_$RANDOM.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/spread/*.json")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["ms_per_step"],4), {k:round(v,4) for k,v in d["kernels_ms"].items()} if "kernels_ms" in d else "")
PY
