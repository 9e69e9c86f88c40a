#!/usr/bin/env bash
# Build timing variants of libdpac into tools/variants/: the LQR float d = 20 object is rebuilt
# with extra -D flags and linked with the main build's other objects.
#   bash tools/build_variants.sh "trace:-DDPAC_NN_TRACE=1 -DDPAC_TU_TRACE=1" "ring3:-DDPAC_NX_RING=3"
# -> tools/variants/libdpac_<name>.so, loaded with DPAC_LIB=<path>.
set -e
cd "$(dirname "$0")/.."
[ -n "$SKIP_MAKE" ] || make -j8 lib >/dev/null
mkdir -p tools/variants
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ideeppde_actorcritic_amd/csrc -Wno-pass-failed -ffp-contract=off -DDPAC_DIMS=20 -DDPAC_DIMS_EVEN=20 -DDPAC_TU_DOUBLE=0"
OTHERS=$(ls build/obj/*.o | grep -v dpac_eqn_lqr_f32_d20.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc $FLAGS $flags -c deeppde_actorcritic_amd/csrc/dpac_eqn_lqr.hip -o tools/variants/lqr_f32_d20_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libdpac_$name.so \
    tools/variants/lqr_f32_d20_$name.o $OTHERS
done
ls -la tools/variants/*.so
