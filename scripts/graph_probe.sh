#!/bin/bash
# Graph-replay investigation (diagnostics, not product): the regression sequence of
# tests/test_driver.py::test_graph_replay_after_eager_launches under the runtime's default graph
# packet capture, with the product library and with the MZ_ARGCHECK build (prints header/argument
# inconsistencies from the device).  PROBE_LIBS selects the builds (default: "prod argcheck").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=${PC:-1} MZ_GRAPH_ENV_EXPERIMENT=1 DBG_TEST_FINAL=${DBG_TEST_FINAL:-1}
for v in ${PROBE_LIBS:-prod argcheck}; do
  if [ "$v" = prod ]; then unset MZ_LIB_OVERRIDE; else export MZ_LIB_OVERRIDE=$PWD/mazero_amd/_build/variant_$v.so; fi
  timeout -k 10 300 python -u scripts/debug_driver_graph.py ${PROBE_ARGS} > "gpurun_out/graph_$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc"; grep -v "^MZCAPTURE" "gpurun_out/graph_$v.log" | tail -6
  if [ $rc -gt 3 ]; then exit $rc; fi
done
exit 0
