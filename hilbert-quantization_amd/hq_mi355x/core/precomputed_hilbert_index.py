"""Pre-computed overlapping-square Hilbert index on MI355X.

Drop-in for the reference's core/precomputed_hilbert_index.py: same classes, dataclasses, method
names, prints and arithmetic.  The averages come from `hq_precomputed_index` (one workgroup per
image, NumPy's pairwise order, bit-identical float32 values) and the similarity from
`hq_precomputed_similarity` (the reference's float32 NumPy arithmetic and Python scalar typing);
`create_precomputed_indices` / `similarity_matrix` are the batched forms the reference lacks.

Reference behaviour kept on purpose:
* `create_precomputed_index` prints its progress lines (:88-117) and caches by model id;
* `PrecomputedSimilaritySearchEngine.search` builds `SearchResult(model=, similarity_score=,
  level_similarities={})` (:350-354), which the reference's own SearchResult dataclass rejects
  (TypeError) — the drop-in raises the same error whenever a candidate passes the threshold;
* the `>= similarity_threshold` test (:342) compares in float32 when the score is a numpy float32
  (NEP 50), in float64 when it is a Python float.
Index files are written with numpy's .npz (no pickle) instead of the reference's pickle (:218-232).
"""
from __future__ import annotations

import functools
import logging
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import kernels as K
from .._dev import to_dev, to_np, torch
from ..models import QuantizedModel, SearchResult
from .hilbert_mapper import HilbertCurveMapper

logger = logging.getLogger(__name__)


@dataclass
class PrecomputedLevel:
    grid_size: int
    square_size: int
    num_squares: int
    averages: np.ndarray
    square_coordinates: List[Tuple[int, int]]


@dataclass
class PrecomputedIndex:
    model_id: str
    original_shape: Tuple[int, int]
    levels: List[PrecomputedLevel]
    creation_time: float
    total_storage_bytes: int


@functools.lru_cache(maxsize=64)
def _square_coordinates(n: int, g: int, s: int) -> List[Tuple[int, int]]:
    """(start_x, start_y) of each square in output order (:169-204): integer geometry only.  Cached:
    indices of one geometry share the (read-only) list."""
    out = [(c * s, r * s) for r in range(g) for c in range(g)]
    off = s // 2
    if off > 0:
        out += [(c * s + off, r * s + off) for r in range(g - 1) for c in range(g - 1)]
    return out


class PrecomputedHilbertIndexer:
    """core/precomputed_hilbert_index.py:43-261 drop-in."""

    def __init__(self, max_levels: int = 6, min_square_size: int = 2):
        self.max_levels = max_levels
        self.min_square_size = min_square_size
        self.hilbert_mapper = HilbertCurveMapper()
        self._index_cache: Dict[str, PrecomputedIndex] = {}

    # ---- layout ---------------------------------------------------------------------------------
    def _calculate_granularity_levels(self, image_size: int) -> List[Tuple[int, int]]:
        return [(g, s) for (g, s, _, _) in K.precomputed_layout(image_size, self.max_levels, self.min_square_size)]

    def _layout(self, n: int):
        return K.precomputed_layout(n, self.max_levels, self.min_square_size)

    # ---- batched device path --------------------------------------------------------------------
    def create_precomputed_indices(self, images=None, parameters=None, n: Optional[int] = None):
        """Batched: images [N, n, n] or Hilbert-ordered parameters [N, d] (with grid side n) ->
        (averages f32 device tensor [N, T], layout [(grid, square, count, first)])."""
        if images is not None:
            x = to_dev(images)
            if x.dim() == 2:
                x = x.view(1, *x.shape)
            side = int(x.shape[-1])
            if int(x.shape[-2]) != side:
                raise ValueError(f"Image must be square, got {int(x.shape[-2])}x{side}")
            return K.precomputed_index(x, side, 0, None, self.max_levels, self.min_square_size), self._layout(side)
        x = to_dev(parameters)
        if n is None:
            raise ValueError("n (grid side) is required for parameter streams")
        return K.precomputed_index(x, int(n), 1, None, self.max_levels, self.min_square_size), self._layout(int(n))

    def _levels_from(self, avg_row: np.ndarray, layout, n: int) -> List[PrecomputedLevel]:
        return [PrecomputedLevel(grid_size=g, square_size=s, num_squares=c, averages=avg_row[o:o + c].copy(),
                                 square_coordinates=_square_coordinates(n, g, s)) for (g, s, c, o) in layout]

    # ---- reference surface ----------------------------------------------------------------------
    def create_precomputed_index(self, image: np.ndarray, model_id: str) -> PrecomputedIndex:
        start_time = time.time()
        height, width = image.shape
        if height != width:
            raise ValueError(f"Image must be square, got {height}x{width}")
        layout = self._layout(width)
        print(f"Pre-computing {len(layout)} granularity levels for {model_id}...")
        avg, _ = self.create_precomputed_indices(images=np.asarray(image))
        row = to_np(avg)[0]
        levels = self._levels_from(row, layout, width)
        total_storage = 0
        for i, lv in enumerate(levels):
            print(f"  Level {i + 1}/{len(levels)}: {lv.grid_size}x{lv.grid_size} grid, "
                  f"{lv.square_size}x{lv.square_size} squares")
            level_storage = lv.averages.nbytes + len(lv.square_coordinates) * 16
            total_storage += level_storage
            print(f"    Computed {lv.num_squares} squares, {level_storage / 1024:.1f} KB")
        creation_time = time.time() - start_time
        index = PrecomputedIndex(model_id=model_id, original_shape=(height, width), levels=levels,
                                 creation_time=creation_time, total_storage_bytes=total_storage)
        self._index_cache[model_id] = index
        print(f"✓ Pre-computed index created in {creation_time:.2f}s")
        print(f"  Total storage: {total_storage / 1024:.1f} KB ({total_storage / (height * width * 4) * 100:.1f}% "
              f"of original)")
        return index

    def _precompute_level_averages(self, image: np.ndarray, grid_size: int, square_size: int) -> PrecomputedLevel:
        n = image.shape[1]
        avg, layout = self.create_precomputed_indices(images=np.asarray(image))
        for lv in self._levels_from(to_np(avg)[0], layout, n):
            if lv.grid_size == grid_size and lv.square_size == square_size:
                return lv
        raise ValueError(f"level ({grid_size}, {square_size}) is not part of the {n}x{n} layout")

    def get_index(self, model_id: str) -> Optional[PrecomputedIndex]:
        return self._index_cache.get(model_id)

    def save_index_to_disk(self, index: PrecomputedIndex, filepath: str):
        arrs = {"model_id": np.array(index.model_id), "original_shape": np.array(index.original_shape),
                "creation_time": np.array(index.creation_time),
                "total_storage_bytes": np.array(index.total_storage_bytes),
                "meta": np.array([[lv.grid_size, lv.square_size, lv.num_squares] for lv in index.levels])}
        for i, lv in enumerate(index.levels):
            arrs[f"avg_{i}"] = lv.averages
            arrs[f"xy_{i}"] = np.array(lv.square_coordinates, dtype=np.int64).reshape(-1, 2)
        with open(filepath, "wb") as f:
            np.savez(f, **arrs)
        logger.info(f"Saved pre-computed index for {index.model_id} to {filepath}")

    def load_index_from_disk(self, filepath: str) -> PrecomputedIndex:
        with np.load(filepath, allow_pickle=False) as z:
            levels = [PrecomputedLevel(int(g), int(s), int(c), z[f"avg_{i}"].copy(),
                                       [tuple(map(int, xy)) for xy in z[f"xy_{i}"]])
                      for i, (g, s, c) in enumerate(z["meta"])]
            index = PrecomputedIndex(str(z["model_id"]), tuple(int(v) for v in z["original_shape"]), levels,
                                     float(z["creation_time"]), int(z["total_storage_bytes"]))
        self._index_cache[index.model_id] = index
        logger.info(f"Loaded pre-computed index for {index.model_id} from {filepath}")
        return index

    def get_storage_overhead(self, original_image_size: int) -> float:
        total = 0
        image_dim = int(np.sqrt(original_image_size // 4))
        for g, s in self._calculate_granularity_levels(image_dim):
            total += (g * g + max(0, (g - 1) * (g - 1))) * (4 + 8)
        return (total / original_image_size) * 100


class PrecomputedSimilaritySearchEngine:
    """core/precomputed_hilbert_index.py:264-512 drop-in (interfaces.SimilaritySearchEngine)."""

    def __init__(self, indexer: PrecomputedHilbertIndexer, similarity_threshold: float = 0.1,
                 level_weights: Optional[List[float]] = None):
        self.indexer = indexer
        self.similarity_threshold = similarity_threshold
        self.level_weights = level_weights or [0.4, 0.3, 0.2, 0.1]

    # ---- weights / level tables (host integer + Python-float plumbing, :390-404) ---------------------
    def _weights(self, n_levels: int) -> List[float]:
        weights = self.level_weights[:n_levels]
        if len(weights) < n_levels:
            remaining = n_levels - len(weights)
            last_weight = weights[-1] if weights else 0.1
            for i in range(remaining):
                weights.append(last_weight * (0.5 ** (i + 1)))
        weight_sum = sum(weights)
        if weight_sum > 0:
            return [w / weight_sum for w in weights]
        return [1.0 / n_levels] * n_levels

    @staticmethod
    def _pack(levels: Sequence[PrecomputedLevel]):
        arr = np.concatenate([np.asarray(lv.averages, dtype=np.float32) for lv in levels]) if levels else \
            np.zeros(0, dtype=np.float32)
        offs, o = [], 0
        for lv in levels:
            offs.append(o)
            o += len(lv.averages)
        return arr, offs

    def similarity_matrix(self, q_avgs, c_avgs, q_offsets, c_offsets, counts, levels: bool = False):
        """Batched device form: query / candidate average rows (same level table) -> (overall f64,
        type u8, level sims) [Q, N] (see kernels.precomputed_similarity)."""
        qa = to_dev(q_avgs, torch().float32)
        ca = to_dev(c_avgs, torch().float32)
        if qa.dim() == 1:
            qa = qa.view(1, -1)
        qs, qn = K.precomputed_stats(qa, q_offsets, counts)
        cs, cn = K.precomputed_stats(ca, c_offsets, counts)
        return K.precomputed_similarity(qa, qn, qs, ca, cn, cs, q_offsets, c_offsets, counts,
                                        self._weights(len(counts)), levels)

    def _pair_tables(self, qi: PrecomputedIndex, ci: PrecomputedIndex):
        L = min(len(qi.levels), len(ci.levels))
        qa, qo = self._pack(qi.levels[:L])
        ca, co = self._pack(ci.levels[:L])
        counts = [min(qi.levels[i].num_squares, ci.levels[i].num_squares) for i in range(L)]
        return qa, ca, qo, co, counts

    @staticmethod
    def _as_reference_type(value: float, kind: int):
        return np.float32(value) if kind == 0 else float(value)

    def _calculate_precomputed_similarity(self, query_index: PrecomputedIndex, candidate_index: PrecomputedIndex):
        if len(query_index.levels) == 0 or len(candidate_index.levels) == 0:
            return 0.0
        qa, ca, qo, co, counts = self._pair_tables(query_index, candidate_index)
        ov, ty, _ = self.similarity_matrix(qa, ca[None], qo, co, counts)
        return self._as_reference_type(float(to_np(ov)[0, 0]), int(to_np(ty)[0, 0]))

    def _compare_precomputed_levels(self, query_level: PrecomputedLevel, candidate_level: PrecomputedLevel):
        if query_level.num_squares == 0 or candidate_level.num_squares == 0:
            return 0.0
        m = min(query_level.num_squares, candidate_level.num_squares)
        qa = np.asarray(query_level.averages, dtype=np.float32)[:m]
        ca = np.asarray(candidate_level.averages, dtype=np.float32)[:m]
        eng = PrecomputedSimilaritySearchEngine(self.indexer, self.similarity_threshold, [1.0])
        _, ty, lv = eng.similarity_matrix(qa, ca[None], [0], [0], [m], levels=True)
        kind = 0 if 0.0 < float(to_np(lv)[0, 0, 0]) < 1.0 and int(to_np(ty)[0, 0]) == 0 else 1
        return self._as_reference_type(float(to_np(lv)[0, 0, 0]), kind)

    def compare_indices_at_level(self, query_indices: np.ndarray, candidate_indices: np.ndarray, level: int) -> float:
        logger.warning("Using legacy comparison method - consider using pre-computed indices for better performance")
        if len(query_indices) == 0 or len(candidate_indices) == 0:
            return 0.0
        m = min(len(query_indices), len(candidate_indices))
        q = to_dev(np.asarray(query_indices, dtype=np.float64)[:m])
        c = to_dev(np.asarray(candidate_indices, dtype=np.float64)[:m].reshape(1, m))
        return float(to_np(K.pearson_f64(q, c))[0])

    def search(self, query_parameters: np.ndarray, candidate_models: List[QuantizedModel],
               max_results: int = 10) -> List[SearchResult]:
        if not candidate_models:
            return []
        query_id = f"query_{hash(query_parameters.tobytes())}"
        query_index = self.indexer.get_index(query_id)
        if query_index is None:
            target_dim = int(np.sqrt(len(query_parameters)))
            if target_dim * target_dim < len(query_parameters):
                target_dim = int(np.ceil(np.sqrt(len(query_parameters))))
                target_dim = 2 ** int(np.ceil(np.log2(target_dim)))
            padded = np.zeros(target_dim * target_dim, dtype=query_parameters.dtype)
            padded[:len(query_parameters)] = query_parameters
            query_image = self.indexer.hilbert_mapper.map_to_2d(padded, (target_dim, target_dim))
            query_index = self.indexer.create_precomputed_index(query_image, query_id)
        # candidates with a cached index, grouped by level table -> one device call per group
        present, groups = [], {}
        for pos, cand in enumerate(candidate_models):
            ci = self.indexer.get_index(cand.metadata.model_name)
            if ci is None:
                logger.warning(f"No pre-computed index found for {cand.metadata.model_name}")
                continue
            present.append(pos)
            key = tuple(lv.num_squares for lv in ci.levels)
            groups.setdefault(key, []).append((pos, ci))
        scores: Dict[int, Tuple[float, int]] = {}
        for members in groups.values():
            if len(query_index.levels) == 0 or len(members[0][1].levels) == 0:
                for pos, _ in members:
                    scores[pos] = (0.0, 1)
                continue
            qa, _, qo, co, counts = self._pair_tables(query_index, members[0][1])
            C = np.stack([self._pair_tables(query_index, ci)[1] for _, ci in members])
            ov, ty, _ = self.similarity_matrix(qa, C, qo, co, counts)
            ov, ty = to_np(ov)[0], to_np(ty)[0]
            for j, (pos, _) in enumerate(members):
                scores[pos] = (float(ov[j]), int(ty[j]))
        similarities = []
        thr = self.similarity_threshold
        for pos in present:
            v, kind = scores[pos]
            passed = (np.float32(v) >= np.float32(thr)) if kind == 0 else (v >= thr)
            if passed:
                similarities.append((self._as_reference_type(v, kind), candidate_models[pos]))
        similarities.sort(key=lambda x: x[0], reverse=True)
        results = []
        for similarity, model in similarities[:max_results]:
            results.append(SearchResult(model=model, similarity_score=similarity, level_similarities={}))
        return results

    def progressive_search(self, query_indices: np.ndarray, candidate_models: List[QuantizedModel],
                           max_results: int = 10) -> List[SearchResult]:
        return self.search(query_indices, candidate_models, max_results)
