set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libikhip_diag.so libikhip_diag_fused.so libikhip_diag.so libikhip_diag_fused.so; do
  IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -k 10 180 python tools/fabrik_diag.py > gpurun_out/diag_${lib}_$RANDOM.json 2>/dev/null || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/diag_*.json")):
    d = json.load(open(f))
    for k, c in d.items():
        print(f.split("/")[-1], k, {x: c[x] for x in ("lane_eff", "steps", "refills", "grabs", "flushes", "refill_us_per_wave", "flush_us_per_wave", "prep_us_per_wave", "wave_dry_us", "wave_end_us")})
PY
REPS=3 TOL=1e-3 MI=100 bash tools/fab_trace_ab.sh libikhip.so libikhip_rf6.so libikhip_rf12.so || exit $?
