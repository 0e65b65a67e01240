"""RAG scoring functions, reference rag/search/engine.py:622-714,1025-1138.

Cosine scores run in hq_cosine_scores; the level weights are host-side constants; multi-level and
windowed scores combine GPU cosine scores exactly like the reference's loops."""
from __future__ import annotations

from typing import List

import numpy as np

from .. import kernels as K
from .._dev import to_dev, to_np


def cosine_scores_batch(a, b):
    """(cos + 1) / 2 of every row of a [Q, K] against every row of b [N, K] -> device f64 [Q, N]."""
    return K.cosine_scores(to_dev(a), to_dev(b))


def calculate_embedding_cosine_similarity(embedding1, embedding2) -> float:
    e1, e2 = np.asarray(embedding1), np.asarray(embedding2)
    if e1.size == 0 or e2.size == 0:
        return 0.0
    f1, f2 = e1.reshape(1, -1).astype(np.float32), e2.reshape(1, -1).astype(np.float32)
    return float(to_np(K.cosine_scores(to_dev(f1), to_dev(f2)))[0, 0])


def compare_single_level_indices(query_indices, candidate_indices) -> float:
    if len(query_indices) == 0 or len(candidate_indices) == 0:
        return 0.0
    return calculate_embedding_cosine_similarity(query_indices, candidate_indices)


def calculate_granularity_weights(num_levels: int) -> np.ndarray:
    if num_levels <= 0:
        return np.array([])
    if num_levels == 1:
        return np.array([1.0])
    w = np.array([8.0 ** (num_levels - i - 1) for i in range(num_levels)])
    w = w / np.sum(w)
    w[0] = w[0] * 2.0
    return w / np.sum(w)


def compare_multi_level_indices(query_indices, candidate_indices) -> float:
    q = np.asarray(query_indices)
    c = np.asarray(candidate_indices)
    levels = q.shape[0]
    if levels == 0:
        return 0.0
    w = calculate_granularity_weights(levels)
    # one GPU launch scores every level pair (row i of q against row i of c)
    s = np.diag(to_np(K.cosine_scores(to_dev(q.astype(np.float32)), to_dev(c.astype(np.float32)))))
    tot, tw = 0.0, 0.0
    for l in range(levels):
        if q.shape[1] == 0 or c.shape[1] == 0:
            continue
        tot += float(s[l]) * w[l]
        tw += w[l]
    return tot / tw if tw else 0.0


def calculate_spatial_locality_similarity(embedding1, embedding2) -> float:
    """4x4 windows at stride 2, mean of windowed cosine (:662-714) on already-extracted images."""
    a, b = np.asarray(embedding1), np.asarray(embedding2)
    if a.shape != b.shape or a.ndim != 2:
        return 0.0
    h, w = a.shape
    ws = min(4, h // 4, w // 4)
    if ws < 2:
        return calculate_embedding_cosine_similarity(a, b)
    wa, wb = [], []
    for i in range(0, h - ws + 1, ws // 2):
        for j in range(0, w - ws + 1, ws // 2):
            wa.append(a[i:i + ws, j:j + ws].ravel())
            wb.append(b[i:i + ws, j:j + ws].ravel())
    if not wa:
        return 0.0
    A = np.stack(wa).astype(np.float32)
    B = np.stack(wb).astype(np.float32)
    s = np.diag(to_np(K.cosine_scores(to_dev(A), to_dev(B))))
    return float(np.mean(s))
