"""Multi-rank root sharding on CPU (gloo, world_size 2 and 4): each rank searches its contiguous shard
of the roots with root_offset; gathered results are bit-identical to one unsharded batch.  Uses
the CPU port as the tree backend, so it runs anywhere; the GPU variant is in test_gpu_parity.py."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PORT_LIB, ROOT, _ensure_oracle_built


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, K, q):
    import ctypes as C
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mazero_amd import _capi
    from mazero_amd.cytree import Tree_batch
    from mazero_amd.shard import max_over_ranks, shard_bounds, slice_inputs
    from mazero_amd.synthetic import make_search_inputs, run_search

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lib = _capi.bind(C.CDLL(PORT_LIB))
    inp = make_search_inputs(np.random.default_rng(42), total, 9, 30)  # same on every rank
    lo, hi = shard_bounds(total, world, rank)
    sub = slice_inputs(inp, lo, hi)
    tb = Tree_batch(hi - lo, 1, 9, K, 30, 0.01, inp.seed, 0.75, 0.8, root_offset=lo, lib=lib)
    out = run_search(tb, sub, K)
    parts = [None] * world
    dist.all_gather_object(parts, {k: out[k] for k in ("sel_idx", "sel_act", "root_values", "marginal_visit_count")})
    mx = max_over_ranks(float(rank + 1), dist)
    if rank == 0:
        full = run_search(Tree_batch(total, 1, 9, K, 30, 0.01, inp.seed, 0.75, 0.8, lib=lib), inp, K)
        ok = mx == float(world)
        for k in ("sel_idx", "sel_act"):
            ok &= np.array_equal(np.concatenate([p[k] for p in parts], axis=1), full[k])
        for k in ("root_values", "marginal_visit_count"):
            ok &= np.array_equal(np.concatenate([p[k] for p in parts], axis=0), full[k])
        q.put(bool(ok))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds():
    from mazero_amd.shard import shard_bounds

    for total in (1, 7, 256, 1000):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(total, world, r) for r in range(world)]
            assert b[0][0] == 0 and b[-1][1] == total
            assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in b) - min(h - l for l, h in b) <= 1


@pytest.mark.parametrize("world,K", [(2, 1), (2, 5), (4, 5)])
def test_gloo_ranks_match_unsharded(world, K):
    """world 4 rehearses a wider job on the CPU: 37 roots split 10/9/9/9 (ragged shards)."""
    _ensure_oracle_built()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 37, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
