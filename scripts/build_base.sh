#!/bin/bash
# Build the product library from a committed revision (default HEAD) into
# mazero_amd/_build/variant_<name>.so, for same-box A/B runs against the working tree's build.
# Usage: scripts/build_base.sh NAME [REV] [-DFOO ...]
cd "$(dirname "$0")/.." || exit 2
name=$1; rev=${2:-HEAD}; shift 2 2>/dev/null
w=.scratch/rev_$name; rm -rf "$w"; mkdir -p "$w"
git archive "$rev" mazero_amd/csrc include | tar -x -C "$w" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -Wno-unused-function -mllvm -amdgpu-kernarg-preload-count=${PRELOAD:-16} \
  -I "$w/include" "$@" "$w/mazero_amd/csrc/mzmcts.hip" "$w/mazero_amd/csrc/mzdriver.hip" "$w/mazero_amd/csrc/mzconsume.hip" \
  -o "mazero_amd/_build/variant_${name}.so" 2>&1 | grep -E "error" ; ls -la "mazero_amd/_build/variant_${name}.so"
