#!/usr/bin/env bash
# Timing variants of libdpac with the MLP TU (dpac_mlp.hip) rebuilt with extra -D flags:
#   tools/build_mlp_variants.sh name:"-DFLAG=1 ..." ...  -> tools/variants/libdpac_<name>.so
set -e
cd "$(dirname "$0")/.."
make -j8 lib >/dev/null
mkdir -p tools/variants
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ideeppde_actorcritic_amd/csrc -Wno-pass-failed -ffp-contract=off"
OTHERS=$(ls build/obj/*.o | grep -v dpac_mlp.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc $HIPFLAGS $flags -c deeppde_actorcritic_amd/csrc/dpac_mlp.hip -o tools/variants/mlp_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libdpac_$name.so tools/variants/mlp_$name.o $OTHERS
done
ls -la tools/variants/*.so
