# Build inversekinematicsann_amd/libikhip_prev.so: the library with the csrc/
# sources of git HEAD, for same-box A/B runs against the working tree
# (tools/fab_ab.sh, tools/ann_ab.sh).
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d /tmp/ikprev.XXXXXX)
trap 'rm -rf $T' EXIT
mkdir -p $T/a/csrc $T/include
REV=${REV:-HEAD}
OUT=${OUT:-libikhip_prev.so}
if [ "$REV" = WORKTREE ]; then  # the working tree's sources (variant builds: EXTRA=-D...)
  cp "$ROOT/include/ikhip.h" $T/include/
  cp "$ROOT"/inversekinematicsann_amd/csrc/*.hip "$ROOT"/inversekinematicsann_amd/csrc/*.h \
     "$ROOT"/inversekinematicsann_amd/csrc/*.cpp $T/a/csrc/
else
  git -C "$ROOT" show $REV:include/ikhip.h > $T/include/ikhip.h
  for f in $(git -C "$ROOT" ls-tree --name-only $REV inversekinematicsann_amd/csrc/); do
    git -C "$ROOT" show $REV:$f > $T/a/csrc/$(basename $f)
  done
fi
cd $T/a/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $EXTRA"
objs=""
for o in ik_fk ik_fabrik ik_ann ik_ann_x ik_ann_w ik_ann_big ik_shard; do
  [ -f $o.hip ] || continue  # (ik_ann_big.hip: r04 on)
  /opt/rocm/bin/hipcc $FLAGS -c $o.hip -o $o.o & objs="$objs $o.o"
done
for o in ik_pipe ik_api; do
  /opt/rocm/bin/hipcc $FLAGS -x hip -c $o.cpp -o $o.o & objs="$objs $o.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/inversekinematicsann_amd/$OUT" $objs
echo "built $OUT from $REV"
