# the r03 and r04 (HEAD) ANN split-mode kernels on ONE box.
# Interleaved runs of tools/ann_ab_min.py (the ABI both builds share) under
# rocprofv3 --kernel-trace --stats, then one GRBM_GUI_ACTIVE pass per build and
# mode for the kernel's clock; tools/ab_split_summary.py prints the table.
# Needs inversekinematicsann_amd/libikhip_r03.so (REV=3abc7e4 OUT=libikhip_r03.so
# bash tools/build_prev.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab_split
mkdir -p $OUT
LIBS=${LIBS:-"libikhip_r03.so libikhip.so"}
MODES=${MODES:-"fp16x3 bf16x6"}
for rep in 1 2; do
  for lib in $LIBS; do
    for mode in $MODES; do
      tag=${lib%.so}__${mode}__t$rep
      timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -- \
        python tools/ann_ab_min.py inversekinematicsann_amd/$lib $mode 20 3 > $OUT/$tag.json 2> $OUT/$tag.err || exit $?
      echo "$tag $(cat $OUT/$tag.json)"
    done
  done
done
for lib in $LIBS; do
  for mode in $MODES; do
    tag=${lib%.so}__${mode}__pmc
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE --output-format csv -d $OUT/$tag -- \
      python tools/ann_ab_min.py inversekinematicsann_amd/$lib $mode 10 3 > $OUT/$tag.json 2> $OUT/$tag.err || exit $?
    echo "$tag $(cat $OUT/$tag.json)"
  done
done
python tools/ab_split_summary.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
