"""Weight broadcast for process-per-GPU self-play (mazero_amd.weights) over gloo, world size 2.

The reference polls a Ray actor for a new checkpoint before each environment step
(selfplay_worker.py:371-375). Here rank 0 publishes a model index and every rank calls sync()
before the step. Checked here:
- the weights arrive bit-identical in the live model, whose parameters are views of the flat
  buffers;
- an unchanged index moves no weights;
- the model still trains and infers afterwards.
The GPU variant (RCCL) runs the same code in tests/test_gpu_parity.py.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mazero_amd.nets import make_net
    from mazero_amd.weights import WeightBroadcaster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    net = make_net(3, 9, seed=100 + rank)  # different weights on every rank
    wb = WeightBroadcaster(net, src=0)
    checks = []
    # nothing published yet: index -1 everywhere, no weight traffic
    checks.append(wb.sync() == -1)
    if rank == 0:
        with torch.no_grad():
            for p in net.parameters():
                p.add_(0.5)
        wb.publish(7)
    checks.append(wb.sync() == 7)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    ref = [None] * world
    dist.all_gather_object(ref, sd)
    checks.append(all(torch.equal(ref[0][k], ref[1][k]) for k in sd))
    # parameters are still views of the flat buffer (a second broadcast lands in the live model)
    flat = wb.flat.tensors()[0]
    p0 = next(net.parameters())
    checks.append(p0.data_ptr() >= flat.data_ptr() and p0.data_ptr() < flat.data_ptr() + flat.numel() * flat.element_size())
    if rank == 0:
        with torch.no_grad():
            p0.mul_(2.0)
    # same index: no weights move (rank 1 keeps its copy)
    wb.sync()
    checks.append((rank == 0) or torch.equal(p0, ref[1][next(iter(sd))]))
    # the model still runs and trains
    out = net.prediction(torch.randn(4, 3 * 128))[0]
    out.sum().backward()
    checks.append(all(p.grad is not None for p in net.policy_head.parameters()))
    q.put((rank, checks))
    dist.barrier()
    dist.destroy_process_group()


def test_flat_weights_preserve_model():
    from mazero_amd.nets import make_net
    from mazero_amd.weights import FlatWeights

    net = make_net(3, 9, seed=1)
    x = torch.randn(5, 3 * 128)
    before = net.prediction(x)[0].detach().clone()
    fw = FlatWeights(net)
    assert fw.numel == sum(p.numel() for p in net.parameters()) + sum(
        b.numel() for b in net.buffers() if b.is_floating_point())
    assert torch.equal(net.prediction(x)[0].detach(), before)


@pytest.mark.timeout(300)
def test_gloo_two_ranks_broadcast():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: [True] * 6, 1: [True] * 6}, res


def _group_worker(rank, world, port, q):
    """World size 4; the broadcast group is global ranks {1, 2, 3} (rank 0, e.g. a learner's peer,
    left out) with the source at global rank 2, group rank 1: the source is named by its global
    rank, as torch.distributed.broadcast takes it (publish compared a group rank
    with it)."""
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mazero_amd.nets import make_net
    from mazero_amd.weights import WeightBroadcaster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grp = dist.new_group([1, 2, 3])  # (every rank takes part in new_group)
    checks = []
    try:
        WeightBroadcaster(make_net(3, 9, seed=1), src=0, group=grp)
        checks.append(False)
    except ValueError:
        checks.append(True)  # a source outside the group is refused
    net = make_net(3, 9, seed=200 + rank)
    if rank != 0:
        wb = WeightBroadcaster(net, src=2, group=grp)
        if rank == 2:
            with torch.no_grad():
                for p in net.parameters():
                    p.add_(0.25)
            wb.publish(5)
        else:
            try:
                wb.publish(5)
                checks.append(False)
            except RuntimeError:
                checks.append(True)  # only the source publishes
        checks.append(wb.sync() == 5)
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    ref = [None] * world
    dist.all_gather_object(ref, sd)
    key = next(iter(sd))
    if rank != 0:
        checks.append(all(torch.equal(ref[2][k], sd[k]) for k in sd))  # the source's weights arrived
    else:
        checks.append(not torch.equal(ref[2][key], sd[key]))  # rank 0 (outside the group) kept its own
    q.put((rank, checks))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_subgroup_broadcast_global_source_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(4))
    for p in procs:
        p.join(timeout=60)
    assert res == {0: [True, True], 1: [True, True, True, True], 2: [True, True, True], 3: [True, True, True, True]}, res


def _rccl_worker(port, q):
    import sys

    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from mazero_amd.nets import make_net
    from mazero_amd.weights import WeightBroadcaster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    net = make_net(3, 9, seed=3, device=torch.device("cuda", 0))
    wb = WeightBroadcaster(net, src=0)
    before = {k: v.clone() for k, v in net.state_dict().items()}
    wb.publish(4)
    ok = wb.sync() == 4 and all(torch.equal(before[k], v) for k, v in net.state_dict().items())
    ok = ok and all(t.is_cuda for t in wb.flat.tensors())
    q.put(bool(ok))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_broadcast_single_rank():
    """The RCCL path (backend "nccl" = RCCL on ROCm) on the device model: flat device buffers,
    index and weights through the collective."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    ok = q.get(timeout=240)
    p.join(timeout=60)
    assert ok


def test_flat_weights_state_dict_keys():
    """FlatWeights holds exactly the floating-point entries of state_dict(): a non-persistent buffer
    stays out (state_dict() lacks it, so load_into(model.state_dict()) works); a
    DistributedDataParallel learner's 'module.'-prefixed state_dict loads too."""
    from mazero_amd.weights import FlatWeights

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(4, 3)
            self.register_buffer("running", torch.zeros(3))
            self.register_buffer("scratch", torch.ones(5), persistent=False)

    src, dst = M(), M()
    with torch.no_grad():
        src.lin.weight.normal_()
        src.running.fill_(2.0)
    fw = FlatWeights(dst)
    assert set(fw.index) == {k for k, v in dst.state_dict().items() if v.is_floating_point()}
    assert "scratch" not in fw.index and fw.numel == 4 * 3 + 3 + 3
    fw.load_into(fw.flats, src.state_dict())
    assert torch.equal(dst.lin.weight, src.lin.weight) and torch.equal(dst.running, src.running)
    with torch.no_grad():
        src.lin.bias.add_(1.0)
    fw.load_into(fw.flats, {"module." + k: v for k, v in src.state_dict().items()})
    assert torch.equal(dst.lin.bias, src.lin.bias)
    with pytest.raises(KeyError):
        fw.load_into(fw.flats, {"lin.weight": src.lin.weight})


def test_counter_only_publish_needs_interval_one():
    """publish(index) without the learner's state_dict makes the live model the checkpoint: fine
    when every new index transfers (interval 1), refused for a longer interval, where the source
    would search newer weights than the other ranks between crossings."""
    import torch.distributed as dist

    from mazero_amd.nets import make_net
    from mazero_amd.weights import WeightBroadcaster

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        net = make_net(3, 9, seed=5)
        wb = WeightBroadcaster(net, src=0, checkpoint_interval=1)
        wb.publish(3)
        assert wb.sync() == 3
        wb10 = WeightBroadcaster(make_net(3, 9, seed=6), src=0, checkpoint_interval=10)
        wb10.publish(0)  # the initial weights are checkpoint 0
        assert wb10.sync() == 0
        with pytest.raises(ValueError, match="state_dict"):
            wb10.publish(12)
        wb10.publish(12, make_net(3, 9, seed=7).state_dict())
        assert wb10.sync() == 12
    finally:
        dist.destroy_process_group()
