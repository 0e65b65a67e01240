"""Tensor-level entry points: one function per C-ABI call of libhq_mi355x (include/hq_mi355x.h).

Inputs and outputs are device tensors (torch on ROCm, used only as HBM buffers); every function
launches HIP kernels on the current stream and never computes on the host.  These are the batched
entry points the reference lacks (`map_to_2d_batch`, `quantize_batch`, `search_batch` in
SURVEY.md §7); the reference-shaped classes in `hq_mi355x.core` / `hq_mi355x.rag` wrap them.
"""
from __future__ import annotations

import functools
import threading

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._dev import device, dtype_code, ptr, stream, torch


def _L():
    return _lib.lib()


def _chk(rc, exc=None):
    _lib.check(rc, exc)


def _contig(x):
    return x if x.is_contiguous() else x.contiguous()


# ---------------------------------------------------------------------------------------------- M


def hilbert_table(n: int, exc=None):
    """(xs, ys, xy2d) int32 device tensors for an n x n grid (core/hilbert_mapper.py:17-113)."""
    t = torch()
    if n <= 0 or (n & (n - 1)) != 0:
        _chk(_L().hq_hilbert_table(n, None, None, None, None), exc)
    xs = t.empty(n * n, dtype=t.int32, device=device())
    ys = t.empty_like(xs)
    tab = t.empty_like(xs)
    _chk(_L().hq_hilbert_table(n, ptr(xs), ptr(ys), ptr(tab), stream()), exc)
    return xs, ys, tab.view(n, n)


def map_to_2d(x, n: int, exc=None):
    """[N, d] (or [d]) -> [N, n, n]: out[y][x] = in[d2xy^-1(x, y)] (core/hilbert_mapper.py:115-174)."""
    t = torch()
    squeeze = x.dim() == 1
    x2 = x.view(1, -1) if squeeze else x
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    N, d = x2.shape
    out = t.empty((N, n, n), dtype=x.dtype, device=x.device)
    _chk(_L().hq_map_to_2d(dtype_code(x.dtype), ptr(x2), N, x2.stride(0) if N > 1 else d, d, n, ptr(out),
                           stream()), exc)
    return out[0] if squeeze else out


def map_from_2d(img, d_out: Optional[int] = None, exc=None):
    """[N, n, n] (or [n, n]) -> [N, d_out] in curve order (core/hilbert_mapper.py:176-205)."""
    t = torch()
    squeeze = img.dim() == 2
    im = _contig(img.unsqueeze(0) if squeeze else img)
    N, n, _ = im.shape
    if d_out is None:
        d_out = n * n
    out = t.empty((N, d_out), dtype=img.dtype, device=img.device)
    _chk(_L().hq_map_from_2d(dtype_code(img.dtype), ptr(im), N, n, d_out, ptr(out), stream()), exc)
    return out[0] if squeeze else out


# ---------------------------------------------------------------------------------------------- I


def index_streaming(img, L: int, stream_len: Optional[int] = None, exc=None):
    """Streaming index of [N, n, n] f32/f64 images -> f64 [N, L] (core/streaming_index_builder.py:315-343).
    The tree covers the first `stream_len` curve positions (default n*n)."""
    t = torch()
    squeeze = img.dim() == 2
    im = _contig(img.unsqueeze(0) if squeeze else img)
    N, n, _ = im.shape
    if stream_len is None:
        stream_len = n * n
    out = t.zeros((N, L), dtype=t.float64, device=im.device)
    _chk(_L().hq_index_streaming(dtype_code(im.dtype), ptr(im), N, n, int(stream_len), L, ptr(out), stream()), exc)
    return out[0] if squeeze else out


def index_traditional(img, L: int, exc=None):
    """Traditional index of [N, n, n] f32 images -> f32 [N, L] (core/index_generator.py:313-356)."""
    t = torch()
    squeeze = img.dim() == 2
    im = _contig((img.unsqueeze(0) if squeeze else img).to(t.float32))
    N, n, _ = im.shape
    out = t.zeros((N, L), dtype=t.float32, device=im.device)
    _chk(_L().hq_index_traditional_f32(ptr(im), N, n, L, ptr(out), stream()), exc)
    return out[0] if squeeze else out


def block_means(img, grid: int, order: int = 0, exc=None):
    """np.mean of each block: order 0 row-major sections, 1 RAG Hilbert order -> f32 [N, cnt]."""
    t = torch()
    squeeze = img.dim() == 2
    im = _contig(img.unsqueeze(0) if squeeze else img)
    if im.dtype not in (t.float32, t.float64):
        im = im.to(t.float32)
    N, n, _ = im.shape
    cnt = 1 if n // grid == 0 else grid * grid
    out = t.empty((N, cnt), dtype=im.dtype, device=im.device)
    _chk(_L().hq_block_means(dtype_code(im.dtype), ptr(im), N, n, int(grid), int(order), ptr(out), stream()), exc)
    return out[0] if squeeze else out


def rag_index_rows(n: int) -> int:
    return _lib.load().hq_rag_index_rows(n)


def index_rag(img, exc=None):
    """RAG multi-row index: [N, n, n] f32 -> [N, n + R, n] (hierarchical_index_generator.py:103-146)."""
    t = torch()
    squeeze = img.dim() == 2
    im = _contig(img.unsqueeze(0) if squeeze else img)
    if im.dtype != t.float32:
        raise TypeError("index_rag: float32 images only")
    N, n, _ = im.shape
    R = rag_index_rows(n)
    out = t.empty((N, n + R, n), dtype=t.float32, device=im.device)
    _chk(_L().hq_index_rag_f32(ptr(im), N, n, ptr(out), stream()), exc)
    return out[0] if squeeze else out


# ---------------------------------------------------------------------------------------------- Q


def quantize_u8(enh, exc=None):
    """[N, r, c] f32 -> (u8 [N, r, c], minmax f32 [N, 2]) (core/compressor.py:256-280)."""
    t = torch()
    squeeze = enh.dim() == 2
    e = _contig(enh.unsqueeze(0) if squeeze else enh)
    N, r, c = e.shape
    out = t.empty((N, r, c), dtype=t.uint8, device=e.device)
    mm = t.empty((N, 2), dtype=t.float32, device=e.device)
    _chk(_L().hq_quantize_u8(ptr(e), N, r, c, ptr(out), ptr(mm), stream()), exc)
    return (out[0], mm[0]) if squeeze else (out, mm)


def dequantize_u8(u8, minmax, exc=None):
    """u8 [N, r, c] with minmax [N, 2] -> f32 (core/compressor.py:282-303)."""
    t = torch()
    squeeze = u8.dim() == 2
    u = _contig(u8.unsqueeze(0) if squeeze else u8)
    mm = _contig(minmax.view(-1, 2).to(t.float32))
    N, r, c = u.shape
    out = t.empty((N, r, c), dtype=t.float32, device=u.device)
    _chk(_L().hq_dequantize_u8(ptr(u), N, r, c, ptr(mm), ptr(out), stream()), exc)
    return out[0] if squeeze else out


def map_index_quantize(x, n: int, L: Optional[int] = None, want_idx: bool = True, want_minmax: bool = True,
                       out: Optional[Tuple] = None, exc=None):
    """The fused north-star kernel: f32 [N, d] -> (u8 frames [N, n+1, n], f64 idx [N, L], f32 minmax [N, 2]).
    Equivalent to pad -> map_to_2d -> streaming index(L) -> embed -> normalise of core/pipeline.py:97-146."""
    t = torch()
    if L is None:
        L = n
    x2 = x if x.dim() == 2 else x.view(1, -1)
    if x2.dtype != t.float32:
        raise TypeError("map_index_quantize expects float32 parameters")
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    N, d = x2.shape
    if out is not None:
        frames, idx, mm = out
    else:
        frames = t.empty((N, n + 1, n), dtype=t.uint8, device=x2.device)
        idx = t.empty((N, L), dtype=t.float64, device=x2.device) if want_idx else None
        mm = t.empty((N, 2), dtype=t.float32, device=x2.device) if want_minmax else None
    _chk(_L().hq_map_index_quantize(ptr(x2), N, x2.stride(0) if N > 1 else d, d, n, L, ptr(frames), ptr(idx),
                                    ptr(mm), stream()), exc)
    return frames, idx, mm


def chunk_encode_f16(x, chunk: int = 1024, exc=None, out=None):
    """Config 5: flat f16 stream -> per-chunk (u8 frame, f32 traditional index, minmax)
    (core/streaming_processor.py:539-582, 877-913).  The last (shorter) chunk uses its own
    geometry inside its slot; unused slot bytes are zero (when `out` is given, the caller's
    buffers are written in place and unused tail-slot bytes are left as they are)."""
    t = torch()
    x1 = _contig(x.reshape(-1))
    if x1.dtype != t.float16:
        raise TypeError("chunk_encode_f16 expects float16")
    total = x1.numel()
    from .core.dimension_calculator import _optimal_side
    ns = _optimal_side(chunk)
    nch = (total + chunk - 1) // chunk
    if out is not None:
        frames, idx, mm = out
        if (tuple(frames.shape) != (nch, ns + 1, ns) or tuple(idx.shape) != (nch, ns) or tuple(mm.shape) != (nch, 2)
                or frames.dtype != t.uint8 or idx.dtype != t.float32 or mm.dtype != t.float32
                or not (frames.is_contiguous() and idx.is_contiguous() and mm.is_contiguous())):
            raise ValueError(f"out buffers must be contiguous u8 [{nch}, {ns + 1}, {ns}], f32 [{nch}, {ns}], "
                             f"f32 [{nch}, 2]")
    else:
        frames = t.zeros((nch, ns + 1, ns), dtype=t.uint8, device=x1.device)
        idx = t.zeros((nch, ns), dtype=t.float32, device=x1.device)
        mm = t.zeros((nch, 2), dtype=t.float32, device=x1.device)
    _chk(_L().hq_chunk_encode_f16(ptr(x1), total, chunk, ptr(frames), ptr(idx), ptr(mm), stream()), exc)
    return frames, idx, mm


# ---------------------------------------------------------------------------------------------- S


def parse_structure(L: int):
    """[(grid, start, end, is_offset)] (core/search_engine.py:42-109), computed by the library."""
    buf = (ctypes.c_int32 * 64)()
    n = _lib.load().hq_parse_structure(int(L), buf, 16)
    return [(buf[4 * i], buf[4 * i + 1], buf[4 * i + 2], bool(buf[4 * i + 3])) for i in range(min(n, 16))]


@functools.lru_cache(maxsize=None)
def seg_count(L: int) -> int:
    return _lib.load().hq_seg_count(int(L))


@functools.lru_cache(maxsize=None)
def seg_level0_len(L: int) -> int:
    return int(_lib.load().hq_seg_level0_len(int(L)))


@functools.lru_cache(maxsize=None)
def seg_padded_len(L: int) -> int:
    return _lib.load().hq_seg_padded_len(int(L))


class Prepared:
    """Device-resident prepared index vectors: raw R [N, L] f64, Z [N, Lp] f64 (segment padded,
    normalised) and stats S [N, nseg, 4] (mean, std, mean of squares, aux).  Built once per corpus.
    f32: some rows are float32 index vectors (aux bit 1; hq_seg_prepare_src / _rows)."""

    __slots__ = ("R", "Z", "S", "L", "N", "nseg", "Lp", "Z16", "S32", "F0", "Zov16", "Sov32", "f32", "all32")

    def __init__(self, R, Z, S, L, f32: bool = False, all32: bool = False):
        self.R, self.Z, self.S, self.L = R, Z, S, int(L)
        self.N = Z.shape[0]
        self.nseg = S.shape[1]
        self.Lp = Z.shape[1]
        self.f32 = bool(f32)      # some rows are float32 sources
        self.all32 = bool(all32)  # every row is
        self.Z16 = self.S32 = None  # split-f16 level-0 copies for the level-0 scan (pack0)
        self.F0 = None  # a corpus's flagged rows of the level-0 copies, listed once (flag_rows)
        self.Zov16 = self.Sov32 = None  # split-f16 copies of every level for the overall scan (packov)

    def rows(self, sel):
        """Sub-set of rows (device index tensor) as a new Prepared (level-0 copies re-packed on demand)."""
        p = Prepared(self.R.index_select(0, sel), self.Z.index_select(0, sel), self.S.index_select(0, sel), self.L,
                     self.f32, self.all32)
        p = pack0(p) if self.Z16 is not None else p
        return packov(p) if self.Zov16 is not None else p

    def unsafe_rows(self):
        """Device bool [N]: float32 rows outside the scans' model (aux bit 2, hq_mi355x.h) -> dense exact path."""
        return (self.S[:, :, 3] >= 2.0).any(dim=1)


def seg_prepare(idx, exc=None, src_f32: bool = False, row_f32=None) -> Prepared:
    """src_f32: every row is a float32 index vector; row_f32 (bool per row, host or device): some are
    (hq_seg_prepare_rows).  The reference computes those rows' statistics and scores in float32."""
    t = torch()
    i2 = _contig((idx if idx.dim() == 2 else idx.view(1, -1)).to(t.float64))
    N, L = i2.shape
    Lp, ns = seg_padded_len(L), seg_count(L)
    Z = t.empty((N, Lp), dtype=t.float64, device=i2.device)
    S = t.empty((N, ns, 4), dtype=t.float64, device=i2.device)
    rf = None
    any32 = all32 = bool(src_f32)
    if row_f32 is not None and not src_f32:
        flags = np.asarray(row_f32, dtype=bool).reshape(-1)
        if flags.size != N:
            raise ValueError("row_f32 needs one flag per row")
        any32, all32 = bool(flags.any()), bool(flags.all()) and N > 0
        rf = _contig(t.from_numpy(flags.astype(np.uint8)).to(i2.device))
    if N:
        _chk(_L().hq_seg_prepare_rows(ptr(i2), N, L, 1 if src_f32 else 0, ptr(rf), ptr(Z), ptr(S), stream()), exc)
    return Prepared(i2, Z, S, L, any32, all32)


PAD0 = 48  # pad rows of the level-0 copies (hq_mi355x.h: hq_seg_pack0_split)


@functools.lru_cache(maxsize=None)
def packov_info(L: int):
    """(K-blocks, G segments, one-value segments, floats per 4-row statistics group) of the split
    overall layout (hq_seg_packov_info), or None when the level structure of L has none."""
    v = [ctypes.c_int() for _ in range(4)]
    if _lib.load().hq_seg_packov_info(int(L), *[ctypes.byref(x) for x in v]) != 0:
        return None
    return tuple(x.value for x in v)


def packov(p: Prepared, exc=None) -> Prepared:
    """Attach the split-f16 copies of every level segment (hq_seg_packov_split) used by the overall
    (brute-force) scan; level structures without a split layout keep the f64 scan."""
    t = torch()
    info = packov_info(p.L)
    if info is None:
        return p
    nkb, _, _, gs = info
    rows = (p.N + 15) // 16 * 16 + PAD0
    p.Zov16 = t.empty((rows, nkb * 64), dtype=t.float16, device=p.Z.device)  # tiled: 16-row tiles of nkb x 2 KiB
    p.Sov32 = t.empty(((p.N + 3) // 4 + PAD0 // 4, gs), dtype=t.float32, device=p.Z.device)  # SoA groups of 4 rows
    _chk(_L().hq_seg_packov_split(ptr(p.Z), ptr(p.S), p.N, p.L, ptr(p.Zov16), ptr(p.Sov32), stream()), exc)
    return p


def pack0(p: Prepared, exc=None) -> Prepared:
    """Attach the split-f16 level-0 copies (hq_seg_pack0_split) used by the level-0 scan; indexes whose
    level-0 segment is longer than 32 values keep the f64 scan."""
    t = torch()
    if seg_level0_len(p.L) > 32:
        return p
    p.Z16 = t.empty(((p.N + 15) // 16 * 16 + PAD0, 64), dtype=t.float16, device=p.Z.device)  # tiled rows
    p.S32 = t.empty(((p.N + 3) // 4 * 4 + PAD0, 4), dtype=t.float32, device=p.Z.device)  # SoA groups of 4 rows
    _chk(_L().hq_seg_pack0_split(ptr(p.Z), ptr(p.S), p.N, p.L, ptr(p.Z16), ptr(p.S32), stream()), exc)
    return p


def seg_prepare_pack0(idx, exc=None, src_f32: bool = False, row_f32=None) -> Prepared:
    """seg_prepare + pack0 in one launch (hq_seg_prepare_pack0): a query batch's statistics, normalised
    rows and split level-0 copies (level-0 segments of <= 32 values; else seg_prepare alone)."""
    t = torch()
    i2 = _contig((idx if idx.dim() == 2 else idx.view(1, -1)).to(t.float64))
    N, L = i2.shape
    if seg_level0_len(L) > 32 or L > 4096:
        return pack0(seg_prepare(i2, exc, src_f32, row_f32), exc)
    Lp, ns = seg_padded_len(L), seg_count(L)
    Z = t.empty((N, Lp), dtype=t.float64, device=i2.device)
    S = t.empty((N, ns, 4), dtype=t.float64, device=i2.device)
    rf = None
    any32 = all32 = bool(src_f32)
    if row_f32 is not None and not src_f32:
        flags = np.asarray(row_f32, dtype=bool).reshape(-1)
        if flags.size != N:
            raise ValueError("row_f32 needs one flag per row")
        any32, all32 = bool(flags.any()), bool(flags.all()) and N > 0
        rf = _contig(t.from_numpy(flags.astype(np.uint8)).to(i2.device))
    p = Prepared(i2, Z, S, L, any32, all32)
    p.Z16 = t.empty(((N + 15) // 16 * 16 + PAD0, 64), dtype=t.float16, device=i2.device)
    p.S32 = t.empty(((N + 3) // 4 * 4 + PAD0, 4), dtype=t.float32, device=i2.device)
    _chk(_L().hq_seg_prepare_pack0(ptr(i2), N, L, 1 if src_f32 else 0, ptr(rf), ptr(Z), ptr(S), ptr(p.Z16),
                                   ptr(p.S32), stream()), exc)
    return p


def flag_rows(p: Prepared, exc=None) -> Prepared:
    """List a corpus's flagged level-0 rows once (hq_seg_flag_rows: int32 [1 + N], count first), so the
    level-0 scan of every query batch skips that pass over the statistics."""
    if p.S32 is None:
        return p
    t = torch()
    p.F0 = t.empty(1 + p.N, dtype=t.int32, device=p.Z.device)
    _chk(_L().hq_seg_flag_rows(ptr(p.S32), p.N, ptr(p.F0), stream()), exc)
    return p


def level_scores(q: Prepared, c: Prepared, level: int, exc=None):
    """Dense EXACT [Q, N] level (>= 0) or overall (level = -1) scores (reference operation order)."""
    t = torch()
    out = t.empty((q.N, c.N), dtype=t.float64, device=q.Z.device)
    _chk(_L().hq_level_scores(ptr(q.R), ptr(q.Z), ptr(q.S), q.N, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L, level,
                              ptr(out), stream()), exc)
    return out


_TLS = threading.local()


def _workspace(nbytes: int, dev):
    """Scan / re-rank workspace reused across the calls ONE thread makes on one stream (stream order
    makes that reuse safe: the previous call's kernels finish before the next call's first write).
    Saves an allocation between the query preparation and the first scan launch of every batch.

    Per thread, not per stream alone: the reference calls its engines from ThreadPoolExecutor workers
    (core/video_search.py:806,854), and threads sharing a stream interleave their launches (ctypes drops
    the GIL), so thread B's scan could otherwise overwrite thread A's workspace between A's scan and A's
    re-rank.  A thread's buffers return to the caching allocator when the thread ends (stream-ordered)."""
    t = torch()
    cache = getattr(_TLS, "ws", None)
    if cache is None:
        cache = _TLS.ws = {}
    key = (str(dev), stream())
    ws = cache.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = cache[key] = t.empty(nbytes, dtype=t.uint8, device=dev)
    return ws[:nbytes]


def scan_topk(q: Prepared, c: Prepared, mode: int, k: int, threshold: float = 0.0, thr_mode: int = 0,
              id_base: int = 0, need_best: bool = False, exc=None):
    """Fused MFMA scan + per-query top-k on APPROXIMATE scores.  mode 0: level-0 score, 1: overall.
    thr_mode 0 none / 1 >= / 2 >.  Returns (scores [Q, k], ids [Q, k], best [Q], best_id [Q]); best and
    best_id (first arg-max of the approximate score) are None unless need_best (the level-0 scan without
    the arg-max runs the wave-independent k_scan0 kernel)."""
    t = torch()
    Q, N = q.N, c.N
    dev = q.Z.device
    ws_bytes = int(_lib.load().hq_scan_workspace_size(Q, N, k))
    ws = _workspace(ws_bytes, dev)
    sc = t.empty((Q, k), dtype=t.float64, device=dev)
    ids = t.empty((Q, k), dtype=t.int64, device=dev)
    best = t.empty(Q, dtype=t.float64, device=dev) if need_best else None
    bid = t.empty(Q, dtype=t.int64, device=dev) if need_best else None
    # option scan_v1 (parity tests): the LDS-tiled k_scan instead of the split-f16 level-0 scan
    if (mode == 0 and not need_best and q.Z16 is not None and c.Z16 is not None
            and (q.f32 or c.f32 or _lib.get_option("scan_v1") is None)):
        _chk(_L().hq_scan0_topk_split_fl(ptr(q.Z16), ptr(q.S32), ptr(q.S), Q, ptr(c.Z16), ptr(c.S32), ptr(c.S), N,
                                         c.L, k, float(threshold), thr_mode, int(id_base), ptr(ws), ws_bytes,
                                         ptr(sc), ptr(ids), None if c.F0 is None else ptr(c.F0), stream()), exc)
        return sc, ids, best, bid
    # option scan_v1 (parity tests): the f64 overall scan instead of the split overall scan
    if mode == 1 and not need_best and q.Zov16 is None and c.Zov16 is not None and _lib.get_option("scan_v1") is None:
        packov(q, exc)  # query batches get the overall layout only when an overall scan needs it
    if (mode == 1 and not need_best and q.Zov16 is not None and c.Zov16 is not None
            and _lib.get_option("scan_v1") is None):
        ws_bytes = int(_lib.load().hq_scanov_workspace_size(Q, N, k))
        ws = _workspace(ws_bytes, dev)
        _chk(_L().hq_scanov_topk_split(ptr(q.Zov16), ptr(q.Sov32), ptr(q.S), ptr(q.Z), Q, ptr(c.Zov16), ptr(c.Sov32),
                                       ptr(c.S), ptr(c.Z), N, c.L, k, float(threshold), thr_mode, int(id_base), ptr(ws),
                                       ws_bytes, ptr(sc), ptr(ids), stream()), exc)
        return sc, ids, best, bid
    _chk(_L().hq_scan_topk(ptr(q.Z), ptr(q.S), Q, ptr(c.Z), ptr(c.S), N, c.L, mode, k, float(threshold), thr_mode,
                           int(id_base), ptr(ws), ws_bytes, ptr(sc), ptr(ids), ptr(best), ptr(bid), stream()), exc)
    return sc, ids, best, bid


def refine_topk(q: Prepared, c: Prepared, mode: int, cand_score, cand_id, k: int, threshold: float = 0.0,
                thr_mode: int = 0, eps: float = 1e-9, id_base: int = 0, exc=None, redo=None, count_empty: bool = False):
    """Exact re-rank of a scan list -> (scores [Q, k], ids [Q, k], count [Q], resolved [Q]).  redo (device
    int32 [1], optional): set to the number of queries needing the dense path (unresolved, or with
    count_empty, nothing passed)."""
    t = torch()
    Q, kp = cand_id.shape
    dev = cand_id.device
    os_ = t.empty((Q, k), dtype=t.float64, device=dev)
    oi = t.empty((Q, k), dtype=t.int64, device=dev)
    cnt = t.empty(Q, dtype=t.int32, device=dev)
    res = t.empty(Q, dtype=t.int32, device=dev)
    if kp > 64:  # long lists: the lane-cooperative re-rank with its workspace
        _refine_ws(q, c, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, os_, oi, cnt, res,
                   count_empty, redo, None, None, exc)
        return os_, oi, cnt, res
    _chk(_L().hq_refine_topk(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L, mode,
                             ptr(_contig(cand_score)), ptr(_contig(cand_id)), kp, k, float(threshold), thr_mode,
                             float(eps), int(id_base), ptr(os_), ptr(oi), ptr(cnt), ptr(res), 1 if count_empty else 0,
                             ptr(redo), stream()), exc)
    return os_, oi, cnt, res


def _refine_ws(q, c, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, os_, oi, cnt, res,
               count_empty, redo, next_redo, det, exc):
    """hq_refine_topk_ws (lists > 64: k_rank_pairs + k_rank_sort) on the stream's reusable workspace (the
    scan that produced the list has finished with it in stream order)."""
    Q = int(cand_id.shape[0])
    dev = cand_id.device
    wb = int(_lib.load().hq_refine_workspace_size(Q, kp, c.L))
    ws = _workspace(wb, dev)
    _chk(_L().hq_refine_topk_ws(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L, mode,
                                ptr(_contig(cand_score)), ptr(_contig(cand_id)), kp, k, float(threshold), thr_mode,
                                float(eps), int(id_base), ptr(os_), ptr(oi), ptr(cnt), ptr(res),
                                1 if count_empty else 0, ptr(redo), ptr(next_redo), ptr(det), ptr(ws), wb, stream()),
         exc)


# refine_final_ws: write the level-0 lists (not returned).  False (the library then skips them, and in round 6 also
# their sort, by selection rounds) measured slower at M = 100 / 1000 (profiles/r06_ab_final_select.txt); the
# selection path was removed, the NULL form kept
FINAL_LEVEL0_LISTS = True


def refine_final_ws(q: Prepared, c: Prepared, cand_score, cand_id, k: int, threshold: float, thr_mode: int,
                    eps: float, id_base: int, K_out: int, redo=None, next_redo=None, exc=None):
    """The level-0 re-rank of a progressive search with its final ranking fused in (hq_refine_final_ws):
    (count, resolved, out_id [Q, K_out], out_det [Q, K_out, 1 + nseg], out_count) as refine_rescore_topk +
    progressive_final with one list and no arg-max fallback; None where the fused form does not exist (the
    caller runs the two steps)."""
    t = torch()
    Q, kp = cand_id.shape
    dev = cand_id.device
    # support probe: with Q = 0 and no counter the call only checks the form exists (nothing launched)
    rc = _L().hq_refine_final_ws(None, None, None, 0, None, None, None, c.N, c.L, None, None, kp, k, 0.0, 0, 0.0, 0,
                                 None, None, None, None, None, None, int(K_out), None, None, None, None, 0, stream())
    if rc == _lib.HQ_E_UNSUPPORTED:
        return None
    _chk(rc, exc)
    # the level-0 lists are not returned (FINAL_LEVEL0_LISTS False: not written)
    os_ = t.empty((Q, k), dtype=t.float64, device=dev) if FINAL_LEVEL0_LISTS else None
    oi = t.empty((Q, k), dtype=t.int64, device=dev) if FINAL_LEVEL0_LISTS else None
    cnt = t.empty(Q, dtype=t.int32, device=dev)
    res = t.empty(Q, dtype=t.int32, device=dev)
    fid = t.empty((Q, K_out), dtype=t.int64, device=dev)
    fdet = t.empty((Q, K_out, 1 + q.nseg), dtype=t.float64, device=dev)
    fcnt = t.empty(Q, dtype=t.int32, device=dev)
    ws, wb = None, 0
    if kp > 64:  # lists <= 64 take k_rank_small, which needs no workspace
        wb = int(_lib.load().hq_refine_workspace_size(Q, kp, c.L))
        ws = _workspace(wb, dev)
    rc = _L().hq_refine_final_ws(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L,
                                 ptr(_contig(cand_score)), ptr(_contig(cand_id)), kp, k, float(threshold), thr_mode,
                                 float(eps), int(id_base), ptr(os_), ptr(oi), ptr(cnt), ptr(res), ptr(redo),
                                 ptr(next_redo), int(K_out), ptr(fid), ptr(fdet), ptr(fcnt), ptr(ws), wb,
                                 stream())
    if rc == _lib.HQ_E_UNSUPPORTED:
        return None
    _chk(rc, exc)
    return cnt, res, fid, fdet, fcnt


def refine_rescore_topk(q: Prepared, c: Prepared, mode: int, cand_score, cand_id, k: int, threshold: float = 0.0,
                        thr_mode: int = 0, eps: float = 1e-9, id_base: int = 0, exc=None, redo=None,
                        count_empty: bool = False, next_redo=None):
    """refine_topk + the exact [overall, level_0..] re-score of its output (rescore's values for the output
    ids, zeros in empty slots) -> (scores, ids, count, resolved, det [Q, k, 1 + nseg])."""
    t = torch()
    Q, kp = cand_id.shape
    dev = cand_id.device
    os_ = t.empty((Q, k), dtype=t.float64, device=dev)
    oi = t.empty((Q, k), dtype=t.int64, device=dev)
    cnt = t.empty(Q, dtype=t.int32, device=dev)
    res = t.empty(Q, dtype=t.int32, device=dev)
    det = t.empty((Q, k, 1 + q.nseg), dtype=t.float64, device=dev)
    if kp > 64:  # long lists: the lane-cooperative re-rank with its workspace
        _refine_ws(q, c, mode, cand_score, cand_id, kp, k, threshold, thr_mode, eps, id_base, os_, oi, cnt, res,
                   count_empty, redo, next_redo, det, exc)
        return os_, oi, cnt, res, det
    if next_redo is not None:  # ping-pong counters: redo arrives zeroed, the kernel clears next_redo
        _chk(_L().hq_refine_rescore_topk_pp(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L,
                                            mode, ptr(_contig(cand_score)), ptr(_contig(cand_id)), kp, k,
                                            float(threshold), thr_mode, float(eps), int(id_base), ptr(os_), ptr(oi),
                                            ptr(cnt), ptr(res), 1 if count_empty else 0, ptr(redo), ptr(next_redo),
                                            ptr(det), stream()), exc)
        return os_, oi, cnt, res, det
    _chk(_L().hq_refine_rescore_topk(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L, mode,
                                     ptr(_contig(cand_score)), ptr(_contig(cand_id)), kp, k, float(threshold),
                                     thr_mode, float(eps), int(id_base), ptr(os_), ptr(oi), ptr(cnt), ptr(res),
                                     1 if count_empty else 0, ptr(redo), ptr(det), stream()), exc)
    return os_, oi, cnt, res, det


def rescore(q: Prepared, c: Prepared, ids, id_base: int = 0, exc=None):
    """EXACT [overall, level_0..] for (query, global id) pairs in ids [Q, k] -> f64 [Q, k, 1 + nseg]."""
    t = torch()
    ids = _contig(ids.to(t.int64))
    Q, k = ids.shape
    out = t.empty((Q, k, 1 + q.nseg), dtype=t.float64, device=ids.device)
    _chk(_L().hq_rescore(ptr(q.R), ptr(q.Z), ptr(q.S), Q, ptr(c.R), ptr(c.Z), ptr(c.S), c.N, c.L, ptr(ids), k,
                         int(id_base), ptr(out), stream()), exc)
    return out


THR_KEY32 = 8  # thr_mode bit of the re-rank: float32 sort keys (hq_mi355x.h HQ_THR_KEY32)


def progressive_final(s0, ids, det, best, best_id, best_det, K: int, exc=None, key32: bool = False):
    """R-way final stage of progressive search.  s0/ids [R, Q, M], det [R, Q, M, W], best/best_id
    [R, Q], best_det [R, Q, W].  Returns (out_id [Q, K], out_det [Q, K, W], count [Q]).  key32: every
    vector is float32, so scores rank by their float32-rounded values (hq_progressive_final_ex flag 1)."""
    t = torch()
    R, Q, M = ids.shape
    W = det.shape[-1]
    dev = ids.device
    oid = t.empty((Q, K), dtype=t.int64, device=dev)
    odet = t.empty((Q, K, W), dtype=t.float64, device=dev)
    cnt = t.empty(Q, dtype=t.int32, device=dev)
    _chk(_L().hq_progressive_final_ex(R, Q, M, W - 1, ptr(_contig(s0)), ptr(_contig(ids)), ptr(_contig(det)),
                                      ptr(_contig(best)), ptr(_contig(best_id)), ptr(_contig(best_det)), K, ptr(oid),
                                      ptr(odet), ptr(cnt), 1 if key32 else 0, stream()), exc)
    return oid, odet, cnt


def cosine_scores_f64(a, b, exc=None):
    """(cos + 1) / 2 of rows of a [Q, K] against rows of b [N, K] (rag/search/engine.py:622-660)."""
    t = torch()
    a2 = _contig(a.reshape(a.shape[0], -1).to(t.float32))
    b2 = _contig(b.reshape(b.shape[0], -1).to(t.float32))
    K = min(a2.shape[1], b2.shape[1])
    if a2.shape[1] != K:
        a2 = _contig(a2[:, :K])
    if b2.shape[1] != K:
        b2 = _contig(b2[:, :K])
    out = t.empty((a2.shape[0], b2.shape[0]), dtype=t.float64, device=a2.device)
    _chk(_L().hq_cosine_scores(ptr(a2), a2.shape[0], ptr(b2), b2.shape[0], K, ptr(out), stream()), exc)
    return out


def cosine_scores_dt(a, b, exc=None):
    """(cos + 1) / 2 of float32 or float64 rows (hq_cosine_scores_dt; float64 stays float64) -> f64 [Q, N].
    float32 problems large enough for the matrix cores take cosine_scores' split-f16 MFMA path."""
    t = torch()
    a2 = _contig(a.reshape(a.shape[0], -1))
    b2 = _contig(b.reshape(b.shape[0], -1))
    if a2.dtype == t.float32 and b2.dtype == t.float32:
        return cosine_scores(a2, b2, exc)
    a2, b2 = a2.to(t.float64), b2.to(t.float64)
    Kd = min(a2.shape[1], b2.shape[1])
    if a2.shape[1] != Kd:
        a2 = _contig(a2[:, :Kd])
    if b2.shape[1] != Kd:
        b2 = _contig(b2[:, :Kd])
    out = t.empty((a2.shape[0], b2.shape[0]), dtype=t.float64, device=a2.device)
    _chk(_L().hq_cosine_scores_dt(dtype_code(t.float64), ptr(a2), a2.shape[0], ptr(b2), b2.shape[0], Kd, ptr(out),
                                  stream()), exc)
    return out


def select_topk(scores, k: int, threshold: float = 0.0, thr_mode: int = 0, id_base: int = 0, exc=None):
    """Top-k (score desc, id asc) of a dense f64 [Q, N] score matrix + first arg-max."""
    t = torch()
    sc = _contig(scores.to(t.float64))
    Q, N = sc.shape
    dev = sc.device
    os_ = t.empty((Q, k), dtype=t.float64, device=dev)
    oi = t.empty((Q, k), dtype=t.int64, device=dev)
    b = t.empty(Q, dtype=t.float64, device=dev)
    bi = t.empty(Q, dtype=t.int64, device=dev)
    ws_bytes = int(_L().hq_select_workspace_size(Q, N, k))
    ws = t.empty(max(ws_bytes, 1), dtype=t.uint8, device=dev)
    _chk(_L().hq_select_topk_ws(ptr(sc), Q, N, k, float(threshold), thr_mode, int(id_base), ptr(ws), ws_bytes,
                                ptr(os_), ptr(oi), ptr(b), ptr(bi), stream()), exc)
    return os_, oi, b, bi


def pair_scores_raw(q, C, exc=None, q_f32: bool = False, c_f32: bool = False):
    """compare_indices_at_level on raw equal-length segments: q [m] vs C [N, m] -> f64 [N]; q_f32 / c_f32:
    that side holds float32 values (statistics in float32; the whole score when both are)."""
    t = torch()
    q1 = _contig(q.reshape(-1).to(t.float64))
    C2 = _contig(C.to(t.float64))
    N, m = C2.shape
    out = t.empty(N, dtype=t.float64, device=C2.device)
    _chk(_L().hq_pair_scores_raw_src(ptr(q1), ptr(C2), N, m, 1 if q_f32 else 0, 1 if c_f32 else 0, ptr(out),
                                     stream()), exc)
    return out


# ------------------------------------------------------------------- §8f row 3: pre-computed index


def precomputed_layout(n: int, max_levels: int = 6, min_square_size: int = 2, exc=None):
    """[(grid, square, count, first_output)] of core/precomputed_hilbert_index.py:121-212 (library)."""
    buf = (ctypes.c_int32 * 64)()
    k = _L().hq_precomputed_layout(int(n), int(max_levels), int(min_square_size), buf, 16)
    if k < 0:
        _chk(k, exc)
    return [(buf[4 * i], buf[4 * i + 1], buf[4 * i + 2], buf[4 * i + 3]) for i in range(min(k, 16))]


def precomputed_index(x, n: int, kind: int = 0, d: Optional[int] = None, max_levels: int = 6,
                      min_square_size: int = 2, exc=None):
    """Overlapping-square averages f32 [N, T] (core/precomputed_hilbert_index.py:65-212).
    kind 0: x = images [N, n, n] (f32/f64); kind 1: x = 1-D Hilbert-ordered parameters [N, d] (f32/f64),
    zero-padded to n*n and mapped to 2-D first (core/pipeline.py:298-319)."""
    t = torch()
    if kind == 0:
        x2 = _contig(x.view(-1, n * n) if x.dim() != 2 or x.shape[1] != n * n else x)
        dd = n * n
    else:
        x2 = x.view(1, -1) if x.dim() == 1 else x
        if x2.stride(-1) != 1:
            x2 = x2.contiguous()
        dd = int(x2.shape[1]) if d is None else int(d)
    N = int(x2.shape[0])
    lay = precomputed_layout(n, max_levels, min_square_size, exc)
    T = sum(c for (_, _, c, _) in lay)
    out = t.empty((N, T), dtype=t.float32, device=x2.device)
    stride = x2.stride(0) if N > 1 else x2.shape[1]
    _chk(_L().hq_precomputed_index(dtype_code(x2.dtype), int(kind), ptr(x2), N, stride, dd, int(n), int(max_levels),
                                   int(min_square_size), ptr(out), T, stream()), exc)
    return out


def precomputed_stats(avgs, offsets, counts, exc=None):
    """Per row and level: stats f32 [N, nlev, 3] (np.mean, np.std, np.mean(a**2)) and the normalised
    averages [N, T] ((a - mean) / std where std != 0) for the first counts[l] values of each level."""
    t = torch()
    a = _contig(avgs)
    N, T = a.shape
    nlev = len(offsets)
    off = (ctypes.c_int32 * nlev)(*offsets)
    cnt = (ctypes.c_int32 * nlev)(*counts)
    st = t.empty((N, nlev, 3), dtype=t.float32, device=a.device)
    nrm = t.zeros_like(a)
    _chk(_L().hq_precomputed_stats(ptr(a), N, T, nlev, off, cnt, ptr(st), ptr(nrm), stream()), exc)
    return st, nrm


def precomputed_similarity(qa, qn, qs, ca, cn, cs, q_offsets, c_offsets, counts, weights, levels: bool = False,
                           exc=None):
    """_calculate_precomputed_similarity for Q x N pairs -> (overall f64 [Q, N], type u8 [Q, N]
    (0 numpy float32, 1 Python float), level sims f64 [Q, N, nlev] or None)."""
    t = torch()
    Q, N = int(qa.shape[0]), int(ca.shape[0])
    nlev = len(counts)
    ov = t.empty((Q, N), dtype=t.float64, device=qa.device)
    ty = t.empty((Q, N), dtype=t.uint8, device=qa.device)
    lv = t.empty((Q, N, nlev), dtype=t.float64, device=qa.device) if levels else None
    _chk(_L().hq_precomputed_similarity(ptr(qa), ptr(qn), ptr(qs), Q, qa.shape[1], ptr(ca), ptr(cn), ptr(cs), N,
                                        ca.shape[1], nlev, (ctypes.c_int32 * nlev)(*q_offsets),
                                        (ctypes.c_int32 * nlev)(*c_offsets), (ctypes.c_int32 * nlev)(*counts),
                                        (ctypes.c_double * nlev)(*weights), ptr(ov), ptr(ty),
                                        ptr(lv) if lv is not None else None, stream()), exc)
    return ov, ty, lv


def pearson_f64(q, C, exc=None):
    """Legacy compare_indices_at_level of the pre-computed engine (:468-496) for q [m] vs C [N, m]."""
    t = torch()
    q1 = _contig(q.reshape(-1))
    C2 = _contig(C)
    N, m = C2.shape
    out = t.empty(N, dtype=t.float64, device=C2.device)
    _chk(_L().hq_pearson_f64(ptr(q1), ptr(C2), N, m, ptr(out), stream()), exc)
    return out


# --------------------------------------------------------------------- S7 on the matrix cores


class CosRows:
    """Split-f16 rows for the MFMA cosine (hq_cos_prepare): X16 [Np, 2, Kp] f16, inv [Np] f64."""

    __slots__ = ("X16", "inv", "N", "K")

    def __init__(self, X16, inv, N, K):
        self.X16, self.inv, self.N, self.K = X16, inv, int(N), int(K)


def cos_prepare(x, exc=None) -> CosRows:
    t = torch()
    x2 = x.view(1, -1) if x.dim() == 1 else x.reshape(x.shape[0], -1)
    if x2.dtype != t.float32:
        x2 = x2.to(t.float32)
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    N, K = int(x2.shape[0]), int(x2.shape[1])
    Kp = int(_L().hq_cos_padded_k(K))
    Np = int(_L().hq_cos_padded_rows(N))
    X16 = t.empty((max(Np, 1), 2, max(Kp, 1)), dtype=t.float16, device=x2.device)
    inv = t.empty(max(Np, 1), dtype=t.float64, device=x2.device)
    if N:
        _chk(_L().hq_cos_prepare(ptr(x2), N, x2.stride(0) if N > 1 else K, K, ptr(X16), ptr(inv), stream()), exc)
    return CosRows(X16, inv, N, K)


def cosine_scores_mfma(q: CosRows, c: CosRows, exc=None, f32: bool = False):
    """(cos + 1) / 2 of every prepared query row against every prepared frame row -> f64 [Q, N]
    (f32=True: float32 [Q, N], the f64 value rounded once — the reference's own score dtype)."""
    t = torch()
    if q.K != c.K:
        raise ValueError(f"query length {q.K} != frame length {c.K}")
    out = t.empty((q.N, c.N), dtype=t.float32 if f32 else t.float64, device=q.X16.device)
    fn = _L().hq_cos_scores_mfma_f32 if f32 else _L().hq_cos_scores_mfma
    _chk(fn(ptr(q.X16), ptr(q.inv), q.N, ptr(c.X16), ptr(c.inv), c.N, q.K, ptr(out), stream()), exc)
    return out


MFMA_COS_MIN_WORK = 1 << 22


def cosine_scores(a, b, exc=None):
    """(cos + 1) / 2 of every row of a [Q, K] against every row of b [N, K] (rag/search/engine.py:622-660)
    -> f64 [Q, N].  Large problems run on the matrix cores (split-f16 MFMA, within 1e-5 of the
    reference's float32 BLAS result); small ones in the f64 kernel."""
    a2 = a.reshape(a.shape[0], -1)
    b2 = b.reshape(b.shape[0], -1)
    Q, N = int(a2.shape[0]), int(b2.shape[0])
    K = min(int(a2.shape[1]), int(b2.shape[1]))  # the reference truncates to the common length
    if Q * N * max(K, 1) >= MFMA_COS_MIN_WORK and K > 0:
        return cosine_scores_mfma(cos_prepare(a2[:, :K], exc), cos_prepare(b2[:, :K], exc), exc)
    return cosine_scores_f64(a, b, exc)
