# One FABRIK experiment lease: the FABRIK GPU parity tests on the working tree's
# build, then tools/fab_ab.sh over the given libraries (interleaved, as given).
# Usage: bash tools/fab_lease.sh LABEL LIB[:VAR=VAL] ...  -> gpurun_out/LABEL/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
label=$1; shift
mkdir -p gpurun_out/$label
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "fabrik or FABRIK or fk_err or core" --timeout 200 --timeout-method thread > gpurun_out/$label/pytest_fabrik.txt 2>&1 || { tail -5 gpurun_out/$label/pytest_fabrik.txt; exit 1; }
tail -1 gpurun_out/$label/pytest_fabrik.txt
bash tools/fab_ab.sh "$@" > gpurun_out/$label/ab.txt 2>&1 || { cat gpurun_out/$label/ab.txt; exit 1; }
cat gpurun_out/$label/ab.txt
