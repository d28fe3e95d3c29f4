#!/bin/bash
# GPU tests on the product build, then the product against two experiment builds in interleaved
# A/B (scripts/ab_ktree.sh): ALT1 / ALT2 = variant .so names under mazero_amd/_build (default
# variant_old / none).  AB_CONFIGS as for ab_ktree.sh.  A failing step ends the run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
B=$PWD/mazero_amd/_build
if [ -z "$SKIP_PYTEST" ]; then
  STEPS=pytest bash scripts/r3_iter.sh || exit $?
  grep -q " passed" gpurun_out/it/pytest_gpu.log && ! grep -qE "[0-9]+ (failed|error)" gpurun_out/it/pytest_gpu.log || { echo "pytest not green"; exit 1; }
fi
for a in ${ALTS:-${ALT1:-variant_old} $ALT2}; do
  echo "== product vs $a"
  ALT=$B/$a.so bash scripts/ab_ktree.sh || exit $?
done
