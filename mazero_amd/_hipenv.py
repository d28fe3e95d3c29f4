"""HIP runtime settings this package depends on, applied at import, before the runtime initialises.

History.  Earlier in round 1 a captured search graph replayed after a few thousand ordinary kernel
launches ran with corrupted arguments in some of its kernels (tests/test_driver.py::
test_graph_replay_after_eager_launches), and the package then set
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 so that every replay marshalled its arguments afresh.  That
setting doubles the cost of every kernel launch in a graph (measured with scripts/launch.hip: an
empty kernel with k_step's 20 arguments costs 1.72 us per launch with packet capture, 3.75 us
without), which was half of the fused tree kernel's 6.4 us per simulation.

With the current argument layout (14 dwords preloaded into SGPRs by the command processor, the
rest read once from a device Params block) the regression test and a 40-replay stress
(scripts/debug_graph_stress.py, ~8,000 eager launches between replays) pass with packet capture
on, with and without the settings below.  The symptom ("some launches saw wrong arguments") is
that of kernel arguments read stale through the host-data-path write combiner, so the package
keeps the runtime's kernarg HDP-flush workaround on:

    DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1   (no measurable launch cost)

and leaves packet capture at the runtime default.  A user who sets
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 keeps the old, slower behaviour.

The runtime reads these variables once, when it initialises.  If the process initialised HIP
before importing mazero_amd without them, SampledMCTS runs its loop eagerly (GRAPHS_SAFE False).
"""
from __future__ import annotations

import os
import sys

KEY = "DEBUG_CLR_KERNARG_HDP_FLUSH_WA"
KEY_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"


def _hip_initialised() -> bool:
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


_user = os.environ.get(KEY)
_user_capture = os.environ.get(KEY_CAPTURE)
_late = _hip_initialised()
os.environ.setdefault(KEY, "1")
GRAPHS_SAFE = (_user == "1") or (_user_capture == "0") or (_user is None and not _late)
if os.environ.get("MZ_GRAPH_ENV_EXPERIMENT") == "1":  # diagnostics: other runtime settings under test
    GRAPHS_SAFE = True
