"""RAG scoring functions, reference rag/search/engine.py:134-162, 243-287,
604-714, 1025-1138.

Every score runs on the GPU (hq_cosine_scores / hq_cosine_scores_dt / hq_cos_scores_mfma,
hq_spatial_locality, hq_detect_heights, hq_threshold_select); the level weights and the progressive
thresholds are host-side constants computed with the reference's own Python float expressions.  Inputs
keep their dtype: float64 arrays are scored in float64 (the reference's np.dot / np.linalg.norm run in
the input dtype), float32 ones from float32 values."""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

from .. import _lib
from .. import kernels as K
from .._dev import dtype_code, ptr, stream, to_dev, to_np, torch


def _score_dtype(*arrays) -> np.dtype:
    """NumPy's result dtype of np.dot / np.linalg.norm on these arrays: float32 only if all are float32."""
    return np.dtype(np.float32) if all(np.asarray(a).dtype == np.float32 for a in arrays) else np.dtype(np.float64)


def cosine_scores_batch(a, b):
    """(cos + 1) / 2 of every row of a [Q, K] against every row of b [N, K] -> device f64 [Q, N]
    (float32 rows: the split-f16 MFMA kernel for large problems; float64 rows in float64)."""
    t = torch()
    a2, b2 = to_dev(a), to_dev(b)
    if a2.dtype == t.float64 or b2.dtype == t.float64:
        return K.cosine_scores_dt(a2.to(t.float64), b2.to(t.float64))
    return K.cosine_scores(a2, b2)


def calculate_embedding_cosine_similarity(embedding1, embedding2) -> float:
    """engine.py:622-660: flatten, truncate to the common length, (cos + 1) / 2, 0 for a zero norm."""
    e1, e2 = np.asarray(embedding1), np.asarray(embedding2)
    if e1.size == 0 or e2.size == 0:
        return 0.0
    m = min(e1.size, e2.size)
    dt = _score_dtype(e1, e2)
    f1 = e1.reshape(-1)[:m].astype(dt, copy=False).reshape(1, -1)
    f2 = e2.reshape(-1)[:m].astype(dt, copy=False).reshape(1, -1)
    return float(to_np(K.cosine_scores_dt(to_dev(f1), to_dev(f2)))[0, 0])


def compare_single_level_indices(query_indices, candidate_indices) -> float:
    """engine.py:1025-1051 (cosine of two 1-D index rows of equal length)."""
    if len(query_indices) == 0 or len(candidate_indices) == 0:
        return 0.0
    return calculate_embedding_cosine_similarity(query_indices, candidate_indices)


def calculate_granularity_weights(num_levels: int) -> np.ndarray:
    """engine.py:1101-1138: 8^(L-i-1), normalised, the first doubled, re-normalised."""
    if num_levels <= 0:
        return np.array([])
    if num_levels == 1:
        return np.array([1.0])
    w = np.array([8.0 ** (num_levels - i - 1) for i in range(num_levels)])
    w = w / np.sum(w)
    w[0] = w[0] * 2.0
    return w / np.sum(w)


def compare_multi_level_indices(query_indices, candidate_indices) -> float:
    """engine.py:1053-1099: weighted mean of the per-level cosines (one launch scores every level pair)."""
    q = np.asarray(query_indices)
    c = np.asarray(candidate_indices)
    levels = q.shape[0]
    if levels == 0:
        return 0.0
    w = calculate_granularity_weights(levels)
    if q.shape[1] == 0 or c.shape[1] == 0:
        return 0.0
    dt = _score_dtype(q, c)
    s = np.diag(to_np(K.cosine_scores_dt(to_dev(q.astype(dt, copy=False)), to_dev(c[:levels].astype(dt, copy=False)))))
    tot, tw = 0.0, 0.0
    for l in range(levels):
        tot += float(s[l]) * w[l]
        tw += w[l]
    return tot / tw if tw else 0.0


def detect_original_embedding_heights(images) -> np.ndarray:
    """engine.py:134-162 for a batch [N, H, W] (or one [H, W] image) -> int heights [N] (hq_detect_heights)."""
    t = torch()
    x = to_dev(images)
    if x.dtype not in (t.float32, t.float64):
        x = x.to(t.float64)
    x3 = (x.unsqueeze(0) if x.dim() == 2 else x).contiguous()
    N, H, W = x3.shape
    out = t.empty(N, dtype=t.int32, device=x3.device)
    _lib.check(_lib.lib().hq_detect_heights(dtype_code(x3.dtype), ptr(x3), N, H, W, ptr(out), stream()))
    return to_np(out).astype(np.int64)


def detect_original_embedding_height(enhanced_embedding) -> int:
    return int(detect_original_embedding_heights(enhanced_embedding)[0])


def extract_original_embedding(enhanced_embedding) -> np.ndarray:
    """engine.py:604-620: a 1-D input as is, else the rows above the detected index rows."""
    e = np.asarray(enhanced_embedding)
    if e.ndim == 1:
        return e
    return e[:detect_original_embedding_height(e), :]


def spatial_locality_scores(queries, images):
    """_calculate_spatial_locality_similarity of every query image [Q, H, W] against every stored
    enhanced image [N, H, W] -> device f64 [Q, N] (hq_spatial_locality: original heights detected on
    both, windowed cosine, NumPy-order mean)."""
    t = torch()
    q, c = to_dev(queries), to_dev(images)
    dt = t.float64 if (q.dtype == t.float64 or c.dtype == t.float64) else t.float32
    q3 = (q.unsqueeze(0) if q.dim() == 2 else q).to(dt).contiguous()
    c3 = (c.unsqueeze(0) if c.dim() == 2 else c).to(dt).contiguous()
    if q3.shape[1:] != c3.shape[1:]:
        raise ValueError(f"image shapes differ: {tuple(q3.shape[1:])} vs {tuple(c3.shape[1:])}")
    Q, H, W = q3.shape
    N = c3.shape[0]
    out = t.empty((Q, N), dtype=t.float64, device=q3.device)
    _lib.check(_lib.lib().hq_spatial_locality(dtype_code(dt), ptr(q3), Q, ptr(c3), N, H, W, ptr(out), stream()))
    return out


def calculate_spatial_locality_similarity(embedding1, embedding2) -> float:
    """engine.py:662-714 on two enhanced (index rows appended) Hilbert images."""
    a, b = np.asarray(embedding1), np.asarray(embedding2)
    if a.shape != b.shape or a.ndim != 2 or a.size == 0:
        return 0.0
    return float(to_np(spatial_locality_scores(a, b))[0, 0])


# ------------------------------------------------------------------ progressive threshold (:243-287)


def progressive_threshold(level: int, n_candidates: int) -> Tuple[float, int]:
    """The level's score threshold and candidate cap, with the reference's Python float arithmetic."""
    base_threshold = 0.3
    level_factor = 0.1
    threshold = base_threshold + (level_factor * (3 - min(level, 3)))
    threshold = min(threshold, 0.8)
    ratio = 0.3 if level == 0 else (0.5 if level == 1 else 0.7)
    return threshold, max(1, int(n_candidates * ratio))


def progressive_threshold_batch(scores, level: int, ids=None):
    """Device form of _apply_progressive_threshold for Q rows of scores [Q, N] in candidate order:
    -> (ids [Q, cap] (-1 padded), count [Q]) with the candidates passing the level's threshold, first
    `cap` in order (ids[q, i] or the position i)."""
    t = torch()
    s = to_dev(scores).to(t.float64)
    s2 = (s.view(1, -1) if s.dim() == 1 else s).contiguous()
    Q, N = s2.shape
    thr, cap = progressive_threshold(level, N)
    idt = None if ids is None else to_dev(ids).to(t.int64).view(Q, N).contiguous()
    out = t.empty((Q, cap), dtype=t.int64, device=s2.device)
    cnt = t.empty(Q, dtype=t.int64, device=s2.device)
    _lib.check(_lib.lib().hq_threshold_select(ptr(s2), ptr(idt), Q, N, float(thr), cap, ptr(out), ptr(cnt), stream()))
    return out, cnt


def apply_progressive_threshold(candidate_scores: Sequence[Tuple[int, float]], level: int) -> List[int]:
    """Drop-in for engine.py:243-287: [(candidate_index, score), ...] -> the passing candidate indices."""
    if not candidate_scores:
        return []
    ids = np.array([int(i) for i, _ in candidate_scores], dtype=np.int64)
    sc = np.array([float(s) for _, s in candidate_scores], dtype=np.float64)
    out, cnt = progressive_threshold_batch(sc[None], level, ids[None])
    n = int(to_np(cnt)[0])
    return [int(x) for x in to_np(out)[0][:n]]
