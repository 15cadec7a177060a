# Variant libptzba for A/B runs: rebuild one source with extra defines and link it with the tree's other
# objects into pan-tilt-zoom-slam_amd/libptzba_NAME.so (run `make` first).
#   bash tools/build_variant.sh NAME SOURCE.hip "-DFOO=1 -DBAR"
set -e
NAME=$1; SRC=$2; DEFS=$3
D=$(cd "$(dirname "$0")/../pan-tilt-zoom-slam_amd/csrc" && pwd)
EXTRA=""; [ "$SRC" = schur_kernels.hip ] && EXTRA=-fno-slp-vectorize
[ "$SRC" = chol_kernels.hip ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-pass-failed -Wno-unused-variable $EXTRA $DEFS \
  -c "$D/$SRC" -o /tmp/variant_$NAME.o
OBJS=$(ls "$D"/*.o | grep -v "/${SRC%.hip}.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS /tmp/variant_$NAME.o -o "$D/../libptzba_$NAME.so"
echo "built libptzba_$NAME.so"
