# r05 lease U: the whole GPU suite, smoke() and the default bench line at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05u
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r05u/pytest_gpu.txt 2>&1; rc=$?
tail -2 gpurun_out/r05u/pytest_gpu.txt; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05u/smoke.txt 2>&1 || exit $?
tail -1 gpurun_out/r05u/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r05u/bench_default.json 2> gpurun_out/r05u/bench_default.err || exit $?
tail -1 gpurun_out/r05u/bench_default.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v.get('ms_per_step') for k, v in d['secondary'].items()})"
