# r05 lease Q: the FABRIK grab size (IKHIP_FABRIK_CHUNK: queue positions a wave
# takes at once, 64 by default) against the launch tail, same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05q
timeout -k 10 1000 bash tools/fab_ab.sh libikhip.so libikhip.so:IKHIP_FABRIK_CHUNK=48 libikhip.so:IKHIP_FABRIK_CHUNK=32 libikhip.so libikhip.so:IKHIP_FABRIK_CHUNK=48 libikhip.so:IKHIP_FABRIK_CHUNK=32 || exit $?
