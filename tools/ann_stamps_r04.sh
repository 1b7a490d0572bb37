set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stamps
for m in fp16x3 bf16x6; do
  MODE=$m IKHIP_LIB=$PWD/inversekinematicsann_amd/libikhip_diag.so timeout -k 10 120 python tools/ann_stamps.py > gpurun_out/stamps/$m.json 2> gpurun_out/stamps/$m.err || exit $?
done
python tools/stamps_summary.py gpurun_out/stamps/fp16x3.json gpurun_out/stamps/bf16x6.json
