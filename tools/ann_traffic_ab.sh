# ANN fp32 HBM traffic A/B: the production build (tiles claimed
# from a counter, IKHIP_ANN_DYN=1) against a static-stride build (IKHIP_ANN_DYN=0,
# libikhip_dyn0.so from tools/build_prev.sh REV=HEAD EXTRA=-DIKHIP_ANN_DYN=0), each
# under three separate --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC hit / miss) plus a
# GRBM_GUI_ACTIVE clock pass, ANN fp32 only.  Summary: tools/ann_traffic_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/anntraffic
mkdir -p $OUT
BENCH="--method ann --secondary 0 --cpu-seconds 0 --end-to-end 0 --cold 0 --steps 5 --warmup 2"
LIBS=${LIBS:-"libikhip.so libikhip_dyn0.so"}
for lib in $LIBS; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES"; do
    i=$((i+1))
    IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib timeout -s KILL 180 rocprofv3 --kernel-trace \
        --pmc $grp --output-format csv -d $OUT/${lib%.so}_$i -- python bench.py $BENCH \
        > $OUT/${lib%.so}_$i.json 2> $OUT/${lib%.so}_$i.err
    rc=$?
    echo "$lib pass $i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
python tools/ann_traffic_summary.py --dir $OUT --builds $(echo $LIBS | sed "s/\.so//g") > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
