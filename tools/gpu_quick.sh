# quick GPU session: tests (optional) + arbitrary python tools, each under a time limit
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/steps.txt
i=0
for cmd in "$@"; do
  i=$((i+1))
  name=${i}_$(echo "$cmd" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-40)
  timeout -k 10 900 bash -c "$cmd" > gpurun_out/q_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
