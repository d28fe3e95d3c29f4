"""HIP runtime settings this package depends on, applied at import, before the runtime initialises.

DEBUG_CLR_GRAPH_PACKET_CAPTURE=0: with the runtime's default graph "packet capture", a captured
search graph replayed after a few thousand ordinary kernel launches on the same device (eager
searches between two replays, for example) ran with corrupted arguments in some of its kernels:
the searches reported errors (or could differ) although the same graph replayed correctly before
and after.  Disabling packet capture makes every replay marshal its kernel arguments afresh
(tests/test_driver.py::test_graph_replay_after_eager_launches); it costs about 1% of the fused
kernel's per-launch time (6.69 -> 6.78 us, 3m K=1).

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
