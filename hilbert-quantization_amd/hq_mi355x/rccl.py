"""The sharded search's one collective through the C-ABI (include/hq_mi355x.h §8e): an RCCL
communicator created by hq_comm_init_rank and the records all-gather hq_allgather_topk (RCCL over xGMI,
one process per GPU).  A non-Python host binds the same four calls; Python callers
bootstrap the communicator id over an existing torch.distributed group (any backend: the 128 id bytes
travel with broadcast_object_list) and then never touch torch.distributed on the data path.

The reference has no collective (its closest analogue is the thread fan-out + list merge of
core/video_search.py:722-875)."""
from __future__ import annotations

import ctypes

from . import _lib
from ._dev import ptr, stream, torch

COMM_ID_BYTES = 128


def unique_id() -> bytes:
    """A fresh communicator id (rank 0 creates it; every rank needs the same bytes)."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _lib.check(_lib.lib().hq_comm_unique_id(buf))
    return buf.raw


class Communicator:
    """RCCL communicator of `nranks` processes, one GPU each (the current device at construction)."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"communicator id must be {COMM_ID_BYTES} bytes")
        self._uid = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().hq_comm_init_rank(ctypes.byref(h), int(nranks), self._uid, int(rank)))
        self.handle = h
        n, r = ctypes.c_int(), ctypes.c_int()
        _lib.check(_lib.lib().hq_comm_size(h, ctypes.byref(n), ctypes.byref(r)))
        self.nranks, self.rank = n.value, r.value

    @classmethod
    def from_process_group(cls, group=None) -> "Communicator":
        """Bootstrap over an initialised torch.distributed group (collective over its ranks)."""
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(world, rank, obj[0])

    @classmethod
    def single(cls) -> "Communicator":
        """A one-rank communicator (tests, one-GPU runs of the sharded path)."""
        return cls(1, 0, unique_id())

    def all_gather(self, x):
        """[R, *x.shape]: every rank's x (device tensor, same shape on all ranks), rank order; async on the
        current stream (hq_allgather_topk)."""
        t = torch()
        xs = x if x.is_contiguous() else x.contiguous()
        out = t.empty((self.nranks,) + tuple(xs.shape), dtype=xs.dtype, device=xs.device)
        _lib.check(_lib.lib().hq_allgather_topk(self.handle, ptr(xs), ptr(out), xs.numel() * xs.element_size(),
                                                stream()))
        return out

    def close(self):
        if self.handle is not None and self.handle.value:
            _lib.check(_lib.lib().hq_comm_destroy(self.handle))
        self.handle = None
