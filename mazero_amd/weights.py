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
    """The model's parameters and persistent floating-point buffers -- the floating-point entries of
    its state_dict -- re-homed as views of one flat tensor per dtype (in `named_parameters` /
    `named_buffers` order, which is identical on every rank for the same architecture).
    Non-persistent buffers are not weights (state_dict() leaves them out) and stay where they are."""

    def __init__(self, model: torch.nn.Module):
        self.model = model
        mods = list(model.named_modules())
        entries = [(m, n, p, True, f"{mn}.{n}" if mn else n) for mn, m in mods for n, p in m._parameters.items()
                   if p is not None]
        entries += [(m, n, b, False, f"{mn}.{n}" if mn else n) for mn, m in mods for n, b in m._buffers.items()
                    if b is not None and b.is_floating_point() and n not in m._non_persistent_buffers_set]
        by_dtype: Dict[torch.dtype, List] = {}
        for e in entries:
            by_dtype.setdefault(e[2].dtype, []).append(e)
        self.flats: Dict[torch.dtype, torch.Tensor] = {}
        self.index: Dict[str, tuple] = {}  # state_dict key -> (dtype, offset, numel)
        for dtype, es in by_dtype.items():
            total = sum(e[2].numel() for e in es)
            flat = torch.empty(total, dtype=dtype, device=es[0][2].device)
            off = 0
            for mod, name, t, is_param, full in es:
                n = t.numel()
                view = flat[off:off + n].view_as(t)
                view.copy_(t.detach())
                if is_param:
                    mod._parameters[name].data = view
                else:
                    mod._buffers[name] = view
                self.index[full] = (dtype, off, n)
                off += n
            self.flats[dtype] = flat

    def load_into(self, flats: Dict[torch.dtype, torch.Tensor], state_dict) -> None:
        """Copy a state_dict (the learner's weights) into flat buffers laid out like these.  A
        DistributedDataParallel learner's keys carry a 'module.' prefix; it is stripped."""
        if self.index and not set(self.index) & set(state_dict):
            pre = "module."
            if all(k.startswith(pre) for k in state_dict):
                state_dict = {k[len(pre):]: v for k, v in state_dict.items()}
        missing = set(self.index) - set(state_dict)
        if missing:
            raise KeyError(f"state_dict lacks {sorted(missing)[:3]}")
        with torch.no_grad():
            for k, (dtype, off, n) in self.index.items():
                flats[dtype][off:off + n].copy_(torch.as_tensor(state_dict[k]).reshape(-1))

    @property
    def numel(self) -> int:
        return sum(f.numel() for f in self.flats.values())

    def tensors(self) -> List[torch.Tensor]:
        return [self.flats[k] for k in sorted(self.flats, key=str)]


class WeightBroadcaster:
    """Periodic weight broadcast from rank `src`.

    `publish(model_index)` on `src` marks the current weights as checkpoint `model_index` (the
    learner's trained-steps counter, shared_storage.get_counter).  `sync()` is called by every rank
    before an environment step: the newest index goes out first, then the weights, but only when
    the index crossed into a new checkpoint interval since this rank's last weights -- the rule of
    `_update_model_before_step` (selfplay_worker.py:371-375):
    `last_model_index // checkpoint_interval < trained_steps // checkpoint_interval`.
    With checkpoint_interval = 1 every new index brings new weights.  It returns the model index
    of the weights each rank now holds."""

    def __init__(self, model: torch.nn.Module, src: int = 0, group=None, checkpoint_interval: int = 1):
        """`src` is the source's GLOBAL rank, as torch.distributed.broadcast takes it even with a
        `group`; a group (e.g. the learner and the self-play ranks only) must contain it."""
        if checkpoint_interval < 1:
            raise ValueError("checkpoint_interval must be >= 1")
        if group is not None and int(src) not in dist.get_process_group_ranks(group):
            raise ValueError(f"source rank {src} is not in the broadcast group {dist.get_process_group_ranks(group)}")
        self.flat = FlatWeights(model)
        self.src = int(src)
        self.group = group
        self.checkpoint_interval = int(checkpoint_interval)
        dev = next(iter(self.flat.flats.values())).device
        self._idx = torch.full((1,), -1, dtype=torch.int64, device=dev)
        self.model_index = -1
        self.syncs = 0  # weight transfers so far
        self._stage = None  # staged learner weights (source rank)
        self._staged = False

    def publish(self, model_index: int, state_dict=None) -> None:
        """Mark checkpoint `model_index` (SharedStorage.set_weights, core/storage.py:68-80).  With
        `state_dict` (the learner's weights) they are staged and become the live weights -- on this
        rank too -- at the next sync that transfers; without it the live model's current weights
        are the checkpoint.  That is only consistent when every new index transfers
        (checkpoint_interval 1): with a longer interval a learner training the source's live model
        in place would have the source search newer weights than the other ranks until the next
        crossing, so publishing without a state_dict is refused there (index 0, the initial weights
        every rank pulls first, excepted)."""
        if dist.get_rank() != self.src:  # (global ranks on both sides: src is one)
            raise RuntimeError("only the source rank publishes weights")
        if state_dict is None and self.checkpoint_interval > 1 and int(model_index) > 0:
            raise ValueError("publish() needs the learner's state_dict when checkpoint_interval > 1 (the live "
                             "model is not a checkpoint between interval crossings)")
        if state_dict is not None:
            if self._stage is None:
                self._stage = {k: torch.empty_like(v) for k, v in self.flat.flats.items()}
            self.flat.load_into(self._stage, state_dict)
            self._staged = True
        self._idx.fill_(int(model_index))

    def _due(self, new: int) -> bool:
        ci = self.checkpoint_interval
        if self.model_index < 0:
            return new >= 0
        return self.model_index // ci < new // ci

    def sync(self) -> int:
        dist.broadcast(self._idx, src=self.src, group=self.group)
        new = int(self._idx.item())
        if new != self.model_index and self._due(new):  # the same decision on every rank
            if self._staged:
                with torch.no_grad():
                    for k, f in self.flat.flats.items():
                        f.copy_(self._stage[k])
                self._staged = False
            for t in self.flat.tensors():
                dist.broadcast(t, src=self.src, group=self.group)
            self.model_index = new
            self.syncs += 1
        return self.model_index
