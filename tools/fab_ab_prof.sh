# FABRIK A/B by rocprof: for each library (under inversekinematicsann_amd/), the
# FABRIK-only bench at tol 1e-3 and 1e-5 under `rocprofv3 --kernel-trace --stats`,
# printing each kernel's average duration (the iteration kernel's is the figure
# the VERDICT's targets use).  Usage: bash tools/fab_ab_prof.sh OUTDIR LIB ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=$1; shift
mkdir -p $out
for lib in "$@"; do
  tag=$(echo "$lib" | tr -c 'a-zA-Z0-9_.' '_')
  for tm in "1e-3 100" "1e-5 200"; do
    set -- $tm
    export IKHIP_LIB=$PWD/inversekinematicsann_amd/$lib
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tag}_$1 -o run -- python bench.py --method fabrik --steps 40 --warmup 5 --cpu-seconds 0 --secondary 0 --end-to-end 0 --cold 0 --tol $1 --max-iter $2 > $out/${tag}_$1.log 2>&1 || exit $?
    echo "$lib tol=$1 $(python tools/kstats.py $out/${tag}_$1)"
  done
done
