# r06 lease: tools/lease.sh (GPU tests, profile_round, fabrik_diag), then the FABRIK
# VALU split (tools/fabrik_valu_split.sh / .py).  Stops at the first crash.
set -o pipefail
cd $GRAFT_REPO_ROOT
SPREAD=0 bash tools/lease.sh || exit $?
bash tools/fabrik_valu_split.sh || exit $?
python tools/fabrik_valu_split.py gpurun_out/valu gpurun_out/fabrik_diag.json ${LOOP_VALU:-157} --json gpurun_out/valu/valu_split.json
