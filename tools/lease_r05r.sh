# r05 lease R: the layered ANN path's bf16x6 GEMM (annb_gemm_x6_kernel): ANN parity
# (split modes incl. the layered models, the kernel-selection test, the oracle
# comparisons), then the layered probe in fp32 and bf16x6 on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r05r
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "ann" -s > gpurun_out/r05r/pytest_ann.txt 2>&1; rc=$?
tail -3 gpurun_out/r05r/pytest_ann.txt; echo "pytest rc=$rc"
grep -E "max\|d\|" gpurun_out/r05r/pytest_ann.txt | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/ann_big_probe.py 262144 all fp32 > gpurun_out/r05r/probe_fp32.txt 2>&1 || exit $?
timeout -k 10 300 python tools/ann_big_probe.py 262144 all bf16x6 > gpurun_out/r05r/probe_bf16x6.txt 2>&1 || exit $?
cat gpurun_out/r05r/probe_fp32.txt gpurun_out/r05r/probe_bf16x6.txt
