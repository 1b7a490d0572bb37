# r05 lease X: the root-space FABRIK band (ik_fabrik_step.h) -- FABRIK parity, an
# A/B against HEAD's build (libikhip_prev.so, tools/build_prev.sh), then the
# whole GPU suite, smoke() and the default bench line (tools/lease_r05u.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "fabrik or FABRIK or fk_err or core" --timeout 200 --timeout-method thread > gpurun_out/r05x/pytest_fabrik.txt 2>&1 || { tail -5 gpurun_out/r05x/pytest_fabrik.txt; exit 1; }
tail -1 gpurun_out/r05x/pytest_fabrik.txt
bash tools/fab_ab.sh libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so libikhip_prev.so libikhip.so > gpurun_out/r05x/ab.txt 2>&1 || { cat gpurun_out/r05x/ab.txt; exit 1; }
cat gpurun_out/r05x/ab.txt
bash tools/lease_r05u.sh
