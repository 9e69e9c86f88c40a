#!/usr/bin/env bash
# Build timing variants of libdpac (LQR f32 TU rebuilt with extra -D flags) into tools/variants/.
set -e
cd "$(dirname "$0")/.."
make -j8 lib >/dev/null
mkdir -p tools/variants
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ideeppde_actorcritic_amd/csrc -DDPAC_DIMS=4,5,10,20 -DDPAC_DIMS_EVEN=4,10,20 -Wno-pass-failed -ffp-contract=off"
OTHERS=$(ls build/obj/*.o | grep -v dpac_eqn_lqr_f32.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc $HIPFLAGS -DDPAC_TU_DOUBLE=0 $flags -c deeppde_actorcritic_amd/csrc/dpac_eqn_lqr.hip -o tools/variants/lqr_f32_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libdpac_$name.so tools/variants/lqr_f32_$name.o $OTHERS
done
ls -la tools/variants/*.so
