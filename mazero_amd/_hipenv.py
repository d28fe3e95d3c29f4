"""HIP runtime settings this package depends on, applied at import, before the runtime initialises.

DEBUG_CLR_GRAPH_PACKET_CAPTURE=0.  With the runtime's default graph "packet capture", a captured
search graph replayed after a few thousand ordinary kernel launches ran with corrupted arguments
in some of its kernels: agent 1's search of tests/test_driver.py::
test_graph_replay_after_eager_launches reports "search path or value-set capacity exceeded",
reproducibly, while the same sequence without the eager searches between capture and replay, or
with packet capture off, matches the oracle (scripts/debug_driver_graph.py).  It does not depend
on kernel-argument preloading, and the runtime's kernarg HDP-flush workaround
(DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1) does not cure it: an earlier commit relied on that workaround
and the regression test failed again on the next fresh box.  A plain torch graph under similar
churn (scripts/debug_torch_graph.py) replays correctly, so the trigger is specific to this launch
mix; turning packet capture off is the fix that holds.  Every replay then marshals its kernel
arguments afresh; on the 3m K=1 bench that costs 0.4 % of the fused kernel's time (5.566 ->
5.588 us per launch, 1 x MI355X).

The runtime reads the variable once, when it initialises.  If the process initialised HIP before
importing mazero_amd without setting it, search graphs are not safe to replay and SampledMCTS runs
its loop eagerly instead (GRAPHS_SAFE is False).
"""
from __future__ import annotations

import os
import sys

KEY = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"


def _hip_initialised() -> bool:
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


_user = os.environ.get(KEY)
_late = _hip_initialised()
os.environ.setdefault(KEY, "0")
GRAPHS_SAFE = (_user == "0") or (_user is None and not _late)
if os.environ.get("MZ_GRAPH_ENV_EXPERIMENT") == "1":  # diagnostics: other runtime settings under test
    GRAPHS_SAFE = True
