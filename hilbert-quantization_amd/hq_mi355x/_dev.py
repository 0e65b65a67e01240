"""Device-buffer plumbing: NumPy <-> torch (ROCm) tensors.  torch is used only for HBM allocation
and streams; all arithmetic runs in libhq_mi355x kernels."""
from __future__ import annotations

import numpy as np

from . import _lib


def torch():
    import torch as _t
    return _t


def device():
    t = torch()
    if not t.cuda.is_available():
        raise _lib.NativeLibraryError("hq_mi355x needs an MI355X; there is no CPU fallback")
    return t.device("cuda", t.cuda.current_device())


_NP2T = None


def _map():
    global _NP2T
    if _NP2T is None:
        t = torch()
        _NP2T = {np.dtype(np.float32): t.float32, np.dtype(np.float64): t.float64, np.dtype(np.float16): t.float16,
                 np.dtype(np.int8): t.int8, np.dtype(np.uint8): t.uint8, np.dtype(np.int16): t.int16,
                 np.dtype(np.int32): t.int32, np.dtype(np.int64): t.int64, np.dtype(np.bool_): t.bool,
                 np.dtype(np.uint16): t.uint16, np.dtype(np.uint32): t.uint32, np.dtype(np.uint64): t.uint64}
    return _NP2T


def is_tensor(x) -> bool:
    try:
        t = torch()
    except ImportError:
        return False
    return isinstance(x, t.Tensor)


def to_dev(x, dtype=None):
    """NumPy array (or tensor) -> contiguous device tensor (bit copy)."""
    t = torch()
    if isinstance(x, t.Tensor):
        out = x if x.is_cuda else x.to(device())
        if dtype is not None and out.dtype != dtype:
            out = out.to(dtype)
        return out.contiguous()
    a = np.ascontiguousarray(x)
    if a.dtype.byteorder not in ("=", "|"):
        a = a.astype(a.dtype.newbyteorder("="))
    tt = _map().get(a.dtype)
    if tt is None:
        raise TypeError(f"unsupported dtype {a.dtype}")
    host = t.from_numpy(a.view(np.uint8).reshape(-1)).view(tt).reshape(a.shape) if a.size else t.empty(a.shape, dtype=tt)
    out = host.to(device(), non_blocking=False)
    if dtype is not None and out.dtype != dtype:
        out = out.to(dtype)
    return out


def to_np(x, np_dtype=None) -> np.ndarray:
    t = torch()
    if isinstance(x, t.Tensor):
        h = x.detach().to("cpu")
        if h.dtype in (t.uint16, t.uint32, t.uint64):
            a = h.view({t.uint16: t.int16, t.uint32: t.int32, t.uint64: t.int64}[h.dtype]).numpy()
            a = a.view({t.uint16: np.uint16, t.uint32: np.uint32, t.uint64: np.uint64}[h.dtype])
        else:
            a = h.numpy()
    else:
        a = np.asarray(x)
    if np_dtype is not None:
        a = a.view(np_dtype) if a.dtype.itemsize == np.dtype(np_dtype).itemsize else a.astype(np_dtype)
    return a


def dtype_code(dt) -> int:
    """HQ dtype code for a numpy dtype or torch dtype (copy kernels only look at the size)."""
    t = torch()
    if isinstance(dt, t.dtype):
        name = str(dt).replace("torch.", "")
    else:
        name = np.dtype(dt).name
    if name not in _lib.DT:
        raise TypeError(f"unsupported dtype {name}")
    return _lib.DT[name]


def ptr(x) -> int:
    return x.data_ptr() if x is not None else 0


def stream() -> int:
    return _lib.stream_ptr()
