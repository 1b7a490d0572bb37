# Build inversekinematicsann_amd/libikhip_prev.so: the library with ik_fabrik.hip
# (or the file given) from git HEAD, for same-box A/B runs (tools/fab_ab.sh).
set -e
cd "$(dirname "$0")/../inversekinematicsann_amd/csrc"
F=${1:-ik_fabrik}
git show HEAD:inversekinematicsann_amd/csrc/$F.hip > ${F}_prev.hip
trap 'rm -f ${F}_prev.hip' EXIT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c ${F}_prev.hip -o /tmp/${F}_prev.o
objs=""
for o in ik_fk ik_fabrik ik_ann ik_ann_x ik_ann_w ik_shard ik_pipe ik_api; do
  if [ "$o" = "$F" ]; then objs="$objs /tmp/${F}_prev.o"; else objs="$objs $o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libikhip_prev.so $objs
