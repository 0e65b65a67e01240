"""ctypes binding of libhq_mi355x.so (include/hq_mi355x.h).

The library is built in-tree (`make -C hilbert-quantization_amd/csrc`, or `__graft_entry__.build()`)
and loaded from this directory.  There is no fallback: if the library is missing or the process has
no GPU, every product entry point raises instead of computing anything on the CPU.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# HQ_LIB_VARIANT: path of another build of the library (the `make DIAG=1` diagnostics build for A/B tools)
LIB_PATH = os.environ.get("HQ_LIB_VARIANT") or os.path.join(_HERE, "libhq_mi355x.so")

HQ_OK = 0
HQ_E_INVALID = -1
HQ_E_NOT_POW2 = -2
HQ_E_TOO_MANY = -3
HQ_E_HIP = -4
HQ_E_UNSUPPORTED = -5

DT = {"float32": 0, "float64": 1, "float16": 2, "bfloat16": 3, "int8": 4, "uint8": 5, "int16": 6,
      "int32": 7, "int64": 8, "uint16": 6, "uint32": 7, "uint64": 8, "bool": 5}

_c = ctypes
_i = _c.c_int
_i64 = _c.c_int64
_p = _c.c_void_p
_d = _c.c_double
_sz = _c.c_size_t

# name -> (restype, argtypes)
SIGNATURES = {
    "hq_version": (_i, []),
    "hq_last_error": (_c.c_char_p, []),
    "hq_set_option": (_i, [_c.c_char_p, _i64]),
    "hq_reset_option": (_i, [_c.c_char_p]),
    "hq_get_option": (_i, [_c.c_char_p, _c.POINTER(_i64)]),
    "hq_diag_build": (_i, []),
    "hq_diag_violations": (_i, [_c.POINTER(_i64), _c.POINTER(_i)]),
    "hq_cosine_scores_dt": (_i, [_i, _p, _i, _p, _i64, _i, _p, _p]),
    "hq_detect_heights": (_i, [_i, _p, _i64, _i, _i, _p, _p]),
    "hq_spatial_locality": (_i, [_i, _p, _i, _p, _i64, _i, _i, _p, _p]),
    "hq_threshold_select": (_i, [_p, _p, _i, _i64, _d, _i64, _p, _p, _p]),
    "hq_comm_unique_id": (_i, [_p]),
    "hq_comm_init_rank": (_i, [_c.POINTER(_p), _i, _p, _i]),
    "hq_comm_size": (_i, [_p, _c.POINTER(_i), _c.POINTER(_i)]),
    "hq_comm_destroy": (_i, [_p]),
    "hq_allgather_topk": (_i, [_p, _p, _p, _sz, _p]),
    "hq_scan0_geometry": (_i, [_i, _i64, _c.POINTER(_i), _c.POINTER(_i), _c.POINTER(_i64), _c.POINTER(_i64),
                               _c.POINTER(_i64)]),
    "hq_hilbert_table": (_i, [_i, _p, _p, _p, _p]),
    "hq_map_to_2d": (_i, [_i, _p, _i64, _i64, _i, _i, _p, _p]),
    "hq_map_from_2d": (_i, [_i, _p, _i64, _i, _i, _p, _p]),
    "hq_index_streaming": (_i, [_i, _p, _i64, _i, _i, _i, _p, _p]),
    "hq_index_traditional_f32": (_i, [_p, _i64, _i, _i, _p, _p]),
    "hq_rag_index_rows": (_i, [_i]),
    "hq_block_means": (_i, [_i, _p, _i64, _i, _i, _i, _p, _p]),
    "hq_index_rag_f32": (_i, [_p, _i64, _i, _p, _p]),
    "hq_quantize_u8": (_i, [_p, _i64, _i, _i, _p, _p, _p]),
    "hq_dequantize_u8": (_i, [_p, _i64, _i, _i, _p, _p, _p]),
    "hq_map_index_quantize": (_i, [_p, _i64, _i64, _i, _i, _i, _p, _p, _p, _p]),
    "hq_chunk_encode_f16": (_i, [_p, _i64, _i, _p, _p, _p, _p]),
    "hq_parse_structure": (_i, [_i, _p, _i]),
    "hq_seg_count": (_i, [_i]),
    "hq_seg_padded_len": (_i, [_i]),
    "hq_seg_prepare": (_i, [_p, _i64, _i, _p, _p, _p]),
    "hq_seg_prepare_src": (_i, [_p, _i64, _i, _i, _p, _p, _p]),
    "hq_seg_prepare_rows": (_i, [_p, _i64, _i, _i, _p, _p, _p, _p]),
    "hq_level_scores": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _p, _p]),
    "hq_refine_topk": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _p, _p, _i, _i, _d, _i, _d, _i64, _p, _p, _p, _p,
                            _i, _p, _p]),
    "hq_refine_rescore_topk": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _p, _p, _i, _i, _d, _i, _d, _i64, _p, _p,
                                    _p, _p, _i, _p, _p, _p]),
    "hq_refine_rescore_topk_pp": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _p, _p, _i, _i, _d, _i, _d, _i64, _p,
                                       _p, _p, _p, _i, _p, _p, _p, _p]),
    "hq_refine_workspace_size": (_sz, [_i, _i, _i]),
    "hq_refine_topk_ws": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _p, _p, _i, _i, _d, _i, _d, _i64, _p, _p, _p,
                               _p, _i, _p, _p, _p, _p, _sz, _p]),
    "hq_refine_final_ws": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _p, _p, _i, _i, _d, _i, _d, _i64, _p, _p, _p, _p,
                                _p, _p, _i, _p, _p, _p, _p, _sz, _p]),
    "hq_scan_workspace_size": (_sz, [_i, _i64, _i]),
    "hq_seg_level0_len": (_i, [_i]),
    "hq_seg_pack0_split": (_i, [_p, _p, _i64, _i, _p, _p, _p]),
    "hq_seg_prepare_pack0": (_i, [_p, _i64, _i, _i, _p, _p, _p, _p, _p, _p]),
    "hq_scan0_topk_split": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _d, _i, _i64, _p, _sz, _p, _p, _p]),
    "hq_seg_flag_rows": (_i, [_p, _i64, _p, _p]),
    "hq_scan0_topk_split_fl": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _i, _d, _i, _i64, _p, _sz, _p, _p, _p, _p]),
    "hq_seg_packov_info": (_i, [_i, _p, _p, _p, _p]),
    "hq_seg_packov_split": (_i, [_p, _p, _i64, _i, _p, _p, _p]),
    "hq_scanov_workspace_size": (_sz, [_i, _i64, _i]),
    "hq_scanov_topk_split": (_i, [_p, _p, _p, _p, _i, _p, _p, _p, _p, _i64, _i, _i, _d, _i, _i64, _p, _sz, _p, _p,
                                  _p]),
    "hq_scan_topk": (_i, [_p, _p, _i, _p, _p, _i64, _i, _i, _i, _d, _i, _i64, _p, _sz, _p, _p, _p, _p, _p]),
    "hq_rescore": (_i, [_p, _p, _p, _i, _p, _p, _p, _i64, _i, _p, _i, _i64, _p, _p]),
    "hq_progressive_final": (_i, [_i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "hq_progressive_final_ex": (_i, [_i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _i, _p, _p, _p, _i, _p]),
    "hq_cosine_scores": (_i, [_p, _i, _p, _i64, _i, _p, _p]),
    "hq_select_topk": (_i, [_p, _i, _i64, _i, _d, _i, _i64, _p, _p, _p, _p, _p]),
    "hq_select_workspace_size": (_sz, [_i, _i64, _i]),
    "hq_select_topk_ws": (_i, [_p, _i, _i64, _i, _d, _i, _i64, _p, _sz, _p, _p, _p, _p, _p]),
    "hq_pair_scores_raw": (_i, [_p, _p, _i64, _i, _p, _p]),
    "hq_pair_scores_raw_src": (_i, [_p, _p, _i64, _i, _i, _i, _p, _p]),
    "hq_precomputed_layout": (_i, [_i, _i, _i, _p, _i]),
    "hq_precomputed_index": (_i, [_i, _i, _p, _i64, _i64, _i, _i, _i, _i, _p, _i64, _p]),
    "hq_precomputed_stats": (_i, [_p, _i64, _i64, _i, _p, _p, _p, _p, _p]),
    "hq_precomputed_similarity": (_i, [_p, _p, _p, _i, _i64, _p, _p, _p, _i64, _i64, _i, _p, _p, _p, _p, _p, _p,
                                       _p, _p]),
    "hq_pearson_f64": (_i, [_p, _p, _i64, _i, _p, _p]),
    "hq_cos_padded_k": (_i, [_i]),
    "hq_cos_padded_rows": (_i64, [_i64]),
    "hq_cos_prepare": (_i, [_p, _i64, _i64, _i, _p, _p, _p]),
    "hq_cos_scores_mfma": (_i, [_p, _p, _i, _p, _p, _i64, _i, _p, _p]),
    "hq_cos_scores_mfma_f32": (_i, [_p, _p, _i, _p, _p, _i64, _i, _p, _p]),
}

_lock = threading.Lock()
_lib = None


class NativeLibraryError(RuntimeError):
    """The HIP library is missing or failed; no CPU fallback exists."""


def load(path: str = LIB_PATH):
    """Load the shared library (no device needed: used by the CPU export test too)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeLibraryError(
                f"{path} not found: build it with `make -C hilbert-quantization_amd/csrc` "
                "(or __graft_entry__.build()); hq_mi355x has no CPU fallback")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


_gpu_ok = False


def lib():
    """The library, on a process that can run kernels (a GPU must be visible; checked until it is)."""
    global _gpu_ok
    if not _gpu_ok:
        import torch
        if not torch.cuda.is_available():
            raise NativeLibraryError("hq_mi355x needs an MI355X (torch.cuda.is_available() is False); "
                                     "there is no CPU fallback")
        _gpu_ok = True
    return load()


def last_error() -> str:
    l = load()
    msg = l.hq_last_error()
    return msg.decode() if msg else ""


def check(rc: int, exc=None):
    """Raise `exc` (or NativeLibraryError) with the library's message when rc != 0."""
    if rc == HQ_OK:
        return
    msg = last_error()
    if exc is None:
        raise NativeLibraryError(f"libhq_mi355x error {rc}: {msg}")
    raise exc(msg)


def stream_ptr(device=None) -> int:
    """hipStream_t of torch's current stream (the raw-pointer query: a few microseconds less per launch)."""
    import torch
    if device is None:
        raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return raw(torch._C._cuda_getDevice())
    return torch.cuda.current_stream(device).cuda_stream


def set_option(name: str, value: int) -> None:
    """Select a kernel variant (hq_set_option; parity tests / A/B only, process-wide)."""
    check(load().hq_set_option(name.encode(), int(value)))


def reset_option(name: str) -> None:
    check(load().hq_reset_option(name.encode()))


def get_option(name: str):
    """The option's value, or None when it is at its default."""
    v = _c.c_int64(0)
    rc = load().hq_get_option(name.encode(), _c.byref(v))
    if rc < 0:
        check(rc)
    return int(v.value) if rc == 1 else None


class option:
    """Context manager: `with option("fused_generic", 1): ...` runs the block with that kernel variant."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, value

    def __enter__(self):
        self.prev = get_option(self.name)
        set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        if self.prev is None:
            reset_option(self.name)
        else:
            set_option(self.name, self.prev)
        return False
