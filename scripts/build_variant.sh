#!/bin/bash
# Experiment build of the product source with extra defines: scripts/build_variant.sh NAME -DFOO ...
# -> mazero_amd/_build/variant_NAME.so (load with MZ_LIB_OVERRIDE=<path>; diagnostics only)
cd "$(dirname "$0")/.." || exit 2
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -Wno-unused-function -mllvm -amdgpu-kernarg-preload-count=${PRELOAD:-16} -I include "$@" \
  mazero_amd/csrc/mzmcts.hip mazero_amd/csrc/mzdriver.hip mazero_amd/csrc/mzconsume.hip -o "mazero_amd/_build/variant_${name}.so"
