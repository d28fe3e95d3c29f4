"""Weight distribution for process-per-GPU self-play.

The reference keeps the weights in a Ray actor (`SharedStorage.get_weights`, core/storage.py:68-80).
Each self-play worker polls it before every environment step and pulls a fresh state_dict
through the object store when a new checkpoint interval has been reached
(selfplay_worker.py:371-375, `_update_model_before_step`).

Here every rank owns one GPU and the model lives there. The holder of the latest weights (rank
`src`, usually the learner) sends them with one collective. Over RCCL (backend "nccl") the
collective runs over xGMI:
- the model's parameters and buffers are re-homed as views into one flat device buffer per
  dtype, so a broadcast writes straight into the live model (no state_dict, no host copy);
- a 3m MAMuZeroNet has 569,585 parameters, i.e. 2.3 MB: one message, about 15 µs at a link's
  153 GB/s;
- the model index travels in the same call sequence. Every rank first learns whether there is
  anything new, so all ranks always take part in the same collectives.

CPU tests run the same code over gloo with world size 2 (tests/test_weights.py).
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.distributed as dist


class FlatWeights:
    """The model's parameters and floating-point buffers, re-homed as views of one flat tensor per
    dtype (in `named_parameters` / `named_buffers` order, which is identical on every rank for the
    same architecture)."""

    def __init__(self, model: torch.nn.Module):
        self.model = model
        entries = [(m, n, p, True) for m in model.modules() for n, p in m._parameters.items() if p is not None]
        entries += [(m, n, b, False) for m in model.modules() for n, b in m._buffers.items()
                    if b is not None and b.is_floating_point()]
        by_dtype: Dict[torch.dtype, List] = {}
        for e in entries:
            by_dtype.setdefault(e[2].dtype, []).append(e)
        self.flats: Dict[torch.dtype, torch.Tensor] = {}
        for dtype, es in by_dtype.items():
            total = sum(e[2].numel() for e in es)
            flat = torch.empty(total, dtype=dtype, device=es[0][2].device)
            off = 0
            for mod, name, t, is_param in es:
                n = t.numel()
                view = flat[off:off + n].view_as(t)
                view.copy_(t.detach())
                if is_param:
                    mod._parameters[name].data = view
                else:
                    mod._buffers[name] = view
                off += n
            self.flats[dtype] = flat

    @property
    def numel(self) -> int:
        return sum(f.numel() for f in self.flats.values())

    def tensors(self) -> List[torch.Tensor]:
        return [self.flats[k] for k in sorted(self.flats, key=str)]


class WeightBroadcaster:
    """Periodic weight broadcast from rank `src`.

    `publish(model_index)` on `src` marks the current weights as checkpoint `model_index`.
    `sync()` is called by every rank before an environment step: the newest index goes out first,
    then the weights, but only when the index changed since the last sync.  It returns the model
    index each rank now holds."""

    def __init__(self, model: torch.nn.Module, src: int = 0, group=None):
        self.flat = FlatWeights(model)
        self.src = src
        self.group = group
        dev = next(iter(self.flat.flats.values())).device
        self._idx = torch.full((1,), -1, dtype=torch.int64, device=dev)
        self.model_index = -1

    def publish(self, model_index: int) -> None:
        if dist.get_rank(self.group) != self.src:
            raise RuntimeError("only the source rank publishes weights")
        self._idx.fill_(int(model_index))

    def sync(self) -> int:
        dist.broadcast(self._idx, src=self.src, group=self.group)
        new = int(self._idx.item())
        if new != self.model_index:
            for t in self.flat.tensors():
                dist.broadcast(t, src=self.src, group=self.group)
            self.model_index = new
        return self.model_index
