# r05 lease W: the default bench line three times in one lease (run-to-run spread
# on one box), then the FABRIK diagnostic breakdown at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05w
for i in 1 2 3; do
  timeout -k 10 600 python bench.py > gpurun_out/r05w/bench_$i.json 2> gpurun_out/r05w/bench_$i.err || exit $?
  tail -1 gpurun_out/r05w/bench_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($i, round(d['value']/1e6,3), round(d['ms_per_step'],3), round(d['roofline']['frac'],4), {k: round(v.get('ms_per_step'),4) for k, v in d['secondary'].items()})"
done
