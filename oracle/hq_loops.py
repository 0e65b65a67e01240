"""Reference-SHAPED CPU port — TEST / BENCH INFRASTRUCTURE ONLY.

`hq_oracle.py` is vectorised NumPy: a fair "best CPU" baseline, but ~800x faster than the reference
itself.  This module keeps the reference's own algorithmic structure — the per-element Python loops —
so `bench.py` can time the CPU path a reference user actually runs, on the GPU box's host cores:

* the coordinate list rebuilt on every map / inverse call, one `_hilbert_index_to_xy` per cell
  (core/hilbert_mapper.py:17-40, 42-66, 92-113), and the per-element scatter / gather loops
  (:157-161, :196-203);
* the streaming index as one `add_value` per stream value into a 4-ary tree of Python floats
  (core/streaming_index_builder.py:45-102, 154-243), fed from a second `map_from_2d` call (:333);
* the uint8 normalise as NumPy vector ops, as the reference (core/compressor.py:256-280);
* the search as a Python loop over candidates, re-parsing both level structures inside every
  comparison (core/search_engine.py:111-189, 129-130; progressive filter :232-300; re-rank :340-388).

Only `bench.py`'s cpu_baseline leg and tests use it (tests/test_oracle_golden.py checks it against the
vectorised oracle).  Nothing in hq_mi355x imports it.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from . import hq_oracle as O


def d2xy(i: int, n: int) -> Tuple[int, int]:
    """One curve index -> (x, y): the quadrant walk with rotate / flip (core/hilbert_mapper.py:42-113)."""
    x = y = 0
    t = i
    s = 1
    while s < n:
        rx = 1 & (t // 2)
        ry = 1 & (t ^ rx)
        if ry == 0:
            if rx == 1:
                x, y = s - 1 - x, s - 1 - y
            x, y = y, x
        x += s * rx
        y += s * ry
        t //= 4
        s *= 2
    return x, y


def coordinates(n: int) -> List[Tuple[int, int]]:
    """generate_hilbert_coordinates: rebuilt per call, one d2xy per cell (:17-40)."""
    return [d2xy(i, n) for i in range(n * n)]


def map_to_2d(p: np.ndarray, n: int) -> np.ndarray:
    out = np.zeros((n, n), dtype=p.dtype)
    coords = coordinates(n)
    for i in range(min(len(p), n * n)):       # per-element scatter (:157-161)
        x, y = coords[i]
        out[y, x] = p[i]
    return out


def map_from_2d(img: np.ndarray) -> np.ndarray:
    n = img.shape[0]
    coords = coordinates(n)
    out = np.zeros(n * n, dtype=img.dtype)
    for i, (x, y) in enumerate(coords):       # per-element gather (:196-203)
        out[i] = img[y, x]
    return out


def streaming_index(stream: np.ndarray, L: int, max_levels: int = 10) -> np.ndarray:
    """One add per value into per-level lists of Python floats; a level promotes every 4th value
    (`(a + b + c + d) * 0.25` left to right), then the strided per-level sampling."""
    levels: List[List[float]] = [[] for _ in range(max_levels)]
    pending: List[List[float]] = [[] for _ in range(max_levels)]
    for v in stream:
        val = float(v)
        lv = 0
        while lv < max_levels:
            levels[lv].append(val)
            pending[lv].append(val)
            if len(pending[lv]) < 4 or lv + 1 >= max_levels:
                break
            a, b, c, d = pending[lv]
            pending[lv] = []
            val = (a + b + c + d) * 0.25
            lv += 1
    sizes = [len(x) for x in levels if x]
    alloc = O.streaming_allocations(sizes, L)
    out: List[float] = []
    for lvl, a in zip(levels, alloc):
        if a <= 0:
            continue
        if len(lvl) > a:
            step = len(lvl) / a
            out.extend(lvl[int(i * step)] for i in range(a))
        else:
            out.extend(lvl)
    res = np.zeros(L, dtype=np.float64)
    res[:min(L, len(out))] = out[:L]
    return res


def quantize_one(p: np.ndarray, n: int, L: int) -> np.ndarray:
    """pad -> map_to_2d -> map_from_2d -> streaming index -> embed -> uint8 normalise (cfg2 per embedding,
    core/pipeline.py:97-146 without the JPEG)."""
    padded = np.zeros(n * n, dtype=p.dtype)
    padded[:len(p)] = p
    img = map_to_2d(padded, n)
    idx = streaming_index(map_from_2d(img), L)
    enh = O.embed_index_row(img, idx)
    u8, _, _ = O.normalize_u8(enh)
    return u8


def precomputed_one(p: np.ndarray, n: int, max_levels: int = 6, min_square_size: int = 2) -> np.ndarray:
    """pad -> map_to_2d -> create_precomputed_index for one model (api.py:162-173): per level, one
    float(np.mean(square)) per grid square then per overlapping square, each stored as float32
    (core/precomputed_hilbert_index.py:65-212)."""
    padded = np.zeros(n * n, dtype=p.dtype)
    padded[:len(p)] = p
    img = map_to_2d(padded, n)
    out: List[np.float32] = []
    for g, s in O.precomputed_levels(n, max_levels, min_square_size):
        for (x0, y0) in O.precomputed_squares(n, g, s):
            out.append(np.float32(float(np.mean(img[y0:y0 + s, x0:x0 + s]))))
    return np.array(out, dtype=np.float32)


def compare_at_level(q: np.ndarray, c: np.ndarray, level: int) -> float:
    """One (query, candidate) comparison; both level structures are re-parsed per call (:129-130)."""
    ql = O.parse_index_structure(len(q))
    cl = O.parse_index_structure(len(c))
    if level >= len(ql) or level >= len(cl):
        return 0.0
    return float(O.level_similarity(q, c[None], level)[0])


def progressive_search(q: np.ndarray, C: np.ndarray, max_results: int, threshold: float = 0.1, M: int = 20):
    """The reference's candidate loop: level-0 score per candidate, keep >= threshold, stable sort, top M
    (first arg-max if none), then the overall score per survivor and a stable sort."""
    sims = [compare_at_level(q, C[i], 0) for i in range(len(C))]
    keep = [i for i in range(len(C)) if sims[i] >= threshold]
    keep.sort(key=lambda i: sims[i], reverse=True)
    keep = keep[:M] if keep else [int(np.argmax(sims))]
    nl = len(O.parse_index_structure(len(q)))
    scored = []
    for i in keep:
        per = [compare_at_level(q, C[i], lv) for lv in range(nl)]
        w = [1.0 / (lv + 1) for lv in range(nl)]
        scored.append((sum(p * x for p, x in zip(per, w)) / sum(w), i))
    scored.sort(key=lambda t: t[0], reverse=True)
    return [i for _, i in scored[:max_results]]
