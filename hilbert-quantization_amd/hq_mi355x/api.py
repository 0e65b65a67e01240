"""High-level API (reference hilbert_quantization/api.py:27-649) on the MI355X components.

HilbertQuantizer keeps quantize / reconstruct / search and the model registry with the reference's
exception wrapping (QuantizationError / ReconstructionError / SearchError / ValidationError).  The
search uses ProgressiveSimilaritySearchEngine(threshold, max_candidates_per_level = 2 * max_results)
as the reference does (api.py:93-101) and filters results >= threshold (:284-287).
BatchQuantizer keeps the reference surface (quantize_batch / search_batch) on the batched device path:
one fused launch per vector length, one resident corpus per search batch.
"""
from __future__ import annotations

import logging
import time
from typing import List, Optional, Union

import numpy as np

from .config import SystemConfig, create_default_config
from .core.dimension_calculator import PowerOf4DimensionCalculator
from .core.precomputed_hilbert_index import PrecomputedHilbertIndexer, PrecomputedSimilaritySearchEngine
from .core.pipeline import QuantizationPipeline, quantize_batch
from .core.search_engine import IndexCorpus, ProgressiveSimilaritySearchEngine
from .exceptions import (HilbertQuantizationError, QuantizationError, ReconstructionError, SearchError,
                         ValidationError)
from .models import ModelMetadata, QuantizedModel, SearchResult


class HilbertQuantizer:
    """api.py:27-565 drop-in: HilbertQuantizer(config=None, use_precomputed_indexing=True).

    The keyword-only arguments override single config fields (similarity_threshold, max_results,
    compression_quality, min_efficiency_ratio) without building a SystemConfig."""

    def __init__(self, config: Optional[SystemConfig] = None, use_precomputed_indexing: bool = True, *,
                 similarity_threshold: Optional[float] = None, max_results: Optional[int] = None,
                 compression_quality: Optional[float] = None, min_efficiency_ratio: Optional[float] = None):
        self.config = config or create_default_config()
        if similarity_threshold is not None:
            self.config.search.similarity_threshold = similarity_threshold
        if max_results is not None:
            self.config.search.max_results = max_results
        if compression_quality is not None:
            self.config.compression.quality = compression_quality
        if min_efficiency_ratio is not None:
            self.config.quantization.min_efficiency_ratio = min_efficiency_ratio
        self.use_precomputed_indexing = use_precomputed_indexing
        self._pipeline: Optional[QuantizationPipeline] = None
        self._engine: Optional[ProgressiveSimilaritySearchEngine] = None
        self._precomputed_indexer: Optional[PrecomputedHilbertIndexer] = None
        self._precomputed_search_engine: Optional[PrecomputedSimilaritySearchEngine] = None
        self._model_registry: List[QuantizedModel] = []
        self.logger = logging.getLogger(__name__)

    # reference-era attribute names
    @property
    def similarity_threshold(self) -> float:
        return self.config.search.similarity_threshold

    @property
    def max_results(self) -> int:
        return self.config.search.max_results

    @property
    def compression_quality(self) -> float:
        return self.config.compression.quality

    @property
    def min_efficiency_ratio(self) -> float:
        return self.config.quantization.min_efficiency_ratio

    @property
    def quantization_pipeline(self) -> QuantizationPipeline:
        if self._pipeline is None:
            self._pipeline = QuantizationPipeline(
                dimension_calculator=PowerOf4DimensionCalculator(self.min_efficiency_ratio),
                compression_config=self.config.compression)
        return self._pipeline

    @property
    def search_engine(self) -> ProgressiveSimilaritySearchEngine:
        if self._engine is None:
            self._engine = ProgressiveSimilaritySearchEngine(self.similarity_threshold, self.max_results * 2)
        return self._engine

    @property
    def precomputed_indexer(self) -> PrecomputedHilbertIndexer:
        if self._precomputed_indexer is None:
            self._precomputed_indexer = PrecomputedHilbertIndexer()
        return self._precomputed_indexer

    @property
    def precomputed_search_engine(self) -> PrecomputedSimilaritySearchEngine:
        if self._precomputed_search_engine is None:
            self._precomputed_search_engine = PrecomputedSimilaritySearchEngine(
                self.precomputed_indexer, similarity_threshold=self.similarity_threshold)
        return self._precomputed_search_engine

    @staticmethod
    def _validate_parameters(p):
        if not isinstance(p, np.ndarray):
            raise ValidationError("Parameters must be a numpy array")
        if p.size == 0:
            raise ValidationError("Parameters array cannot be empty")
        if p.ndim != 1:
            raise ValidationError("Parameters must be a 1D array")
        if not np.all(np.isfinite(p)):
            raise ValidationError("Parameters contain non-finite values (NaN or infinity)")

    def quantize(self, parameters: Union[np.ndarray, List[float]], model_id: Optional[str] = None,
                 description: Optional[str] = None, validate: bool = True) -> QuantizedModel:
        try:
            if isinstance(parameters, list):
                parameters = np.array(parameters, dtype=np.float32)
            if validate:
                self._validate_parameters(parameters)
            qm = self.quantization_pipeline.quantize_model(parameters, model_id or f"model_{int(time.time())}",
                                                           compression_quality=self.compression_quality,
                                                           model_architecture=description)
            if self.use_precomputed_indexing:  # api.py:162-173
                try:
                    image_2d = self.quantization_pipeline._get_2d_representation(parameters)
                    pre = self.precomputed_indexer.create_precomputed_index(image_2d, qm.metadata.model_name)
                    self.logger.info(f"Pre-computed index created: {pre.total_storage_bytes / 1024:.1f}KB")
                except Exception as e:  # the reference continues without the index
                    self.logger.warning(f"Failed to create pre-computed index: {e}")
            self._model_registry.append(qm)
            return qm
        except (QuantizationError, ValidationError):
            raise
        except Exception as e:
            raise QuantizationError(f"Unexpected error during quantization: {e}") from e

    def quantize_many(self, parameter_sets, model_ids: Optional[List[str]] = None,
                      descriptions: Optional[List[str]] = None, validate: bool = True) -> List[QuantizedModel]:
        """quantize() for many vectors in one batched device pass (same models, registry, indices)."""
        return _ingest(self, parameter_sets, model_ids, descriptions, True, validate)

    def reconstruct(self, quantized_model: QuantizedModel, validate: bool = True) -> np.ndarray:
        try:
            return self.quantization_pipeline.reconstruct_parameters(quantized_model)
        except (ReconstructionError, ValidationError):
            raise
        except Exception as e:
            raise ReconstructionError(f"Unexpected error during reconstruction: {e}") from e

    def reconstruct_many(self, quantized_models: List[QuantizedModel], validate: bool = True) -> List[np.ndarray]:
        """reconstruct() for many models: host JPEG decode on threads, one de-normalise and one inverse
        Hilbert gather per frame shape (core.pipeline.reconstruct_batch); same arrays and errors."""
        from .core.pipeline import reconstruct_batch
        try:
            out = reconstruct_batch(quantized_models, self.quantization_pipeline.compressor)
            return [o if o is not None else self.reconstruct(m, validate) for o, m in zip(out, quantized_models)]
        except (ReconstructionError, ValidationError):
            raise
        except Exception as e:
            raise ReconstructionError(f"Unexpected error during reconstruction: {e}") from e

    def search(self, query_parameters, candidate_models: Optional[List[QuantizedModel]] = None,
               max_results: Optional[int] = None, similarity_threshold: Optional[float] = None) -> List[SearchResult]:
        try:
            if isinstance(query_parameters, list):
                query_parameters = np.array(query_parameters, dtype=np.float32)
            self._validate_parameters(query_parameters)
            candidates = candidate_models or self._model_registry
            if not candidates:
                raise SearchError("No candidate models available for search")
            max_results = max_results or self.max_results
            thr = similarity_threshold or self.similarity_threshold
            query = self.quantize(query_parameters, validate=False)
            results = self.search_engine.progressive_search(query.hierarchical_indices, candidates, max_results)
            return [r for r in results if r.similarity_score >= thr]
        except (SearchError, ValidationError, QuantizationError):
            raise
        except Exception as e:
            raise SearchError(f"Unexpected error during search: {e}") from e

    def get_registry_info(self):
        return {"total_models": len(self._model_registry),
                "model_ids": [m.metadata.model_name for m in self._model_registry]}

    def clear_registry(self):
        self._model_registry.clear()


def _ingest(hq: "HilbertQuantizer", parameter_sets, model_ids=None, descriptions=None, parallel: bool = True,
            validate: bool = True, verbose: bool = False) -> List[QuantizedModel]:
    """Batched HilbertQuantizer.quantize: the same QuantizedModels, registry entries,
    pre-computed indices and compressor state as calling quantize() model by model, in order.

    float32 vectors of one length go through ONE fused launch (hq_map_index_quantize: frames, f64
    indices, min/max) and one pre-computed-index launch; the frames come back in one copy and the host
    JPEG stage (same call as core/compressor.py:71-80, byte-identical output) runs on a thread pool.
    Validation and efficiency failures surface at the same model, with the same exception, as the
    sequential path (models before it are quantized and registered first).  Other dtypes take the
    per-model path.  `verbose` = the reference's per-model pre-computed-index prints."""
    import concurrent.futures as cf
    import os as _os
    from .core.compressor import encode_jpeg
    from .core.precomputed_hilbert_index import PrecomputedIndex, _square_coordinates, PrecomputedLevel
    from ._dev import to_dev, to_np
    from . import kernels as K

    sets = [np.array(p, dtype=np.float32) if isinstance(p, list) else p for p in parameter_sets]
    names = [model_ids[i] if model_ids else f"model_{i}" for i in range(len(sets))]
    descs = [descriptions[i] if descriptions else None for i in range(len(sets))]
    # first failure in sequence order (validation, then dimension / efficiency check)
    stop, stop_exc = len(sets), None
    for i, p in enumerate(sets):
        try:
            if validate:
                hq._validate_parameters(p)
            if p.dtype == np.float32:
                calc = PowerOf4DimensionCalculator(hq.min_efficiency_ratio)
                calc.calculate_padding_strategy(len(p), calc.calculate_optimal_dimensions(len(p)))
        except Exception as e:
            stop = i
            stop_exc = e if isinstance(e, (QuantizationError, ValidationError)) else \
                QuantizationError(f"Unexpected error during quantization: "
                                  f"{HilbertQuantizationError(f'Failed to quantize model {names[i]!r}: {e}')}")
            break
    out: List[Optional[QuantizedModel]] = [None] * stop
    groups = {}
    for i in range(stop):
        if sets[i].dtype == np.float32 and sets[i].ndim == 1:
            groups.setdefault(len(sets[i]), []).append(i)
        else:
            out[i] = None  # per-model path below
    pipe = hq.quantization_pipeline
    quality = hq.compression_quality
    last_state = None  # (position, min, max) of the last non-constant frame: the compressor's state
    workers = min(32, _os.cpu_count() or 1) if parallel else 1
    with cf.ThreadPoolExecutor(max_workers=workers) as pool:
        for d, members in groups.items():
            X = to_dev(np.stack([sets[i] for i in members]))
            frames, idx, mm = quantize_batch(X, hq.min_efficiency_ratio)
            n = int(frames.shape[2])
            pre = K.precomputed_index(X, n, 1) if hq.use_precomputed_indexing else None
            fr_h, idx_h, mm_h = to_np(frames), to_np(idx), to_np(mm)
            jpegs = list(pool.map(lambda k: encode_jpeg(fr_h[k], quality), range(len(members))))
            pre_h = to_np(pre) if pre is not None else None
            layout = K.precomputed_layout(n) if pre is not None else None
            for k, i in enumerate(members):
                data = jpegs[k]
                size = sets[i].nbytes
                md = ModelMetadata(model_name=names[i], original_size_bytes=size, compressed_size_bytes=len(data),
                                   compression_ratio=size / len(data) if data else 0.0,
                                   quantization_timestamp=time.strftime("%Y-%m-%d %H:%M:%S"),
                                   model_architecture=descs[i], additional_info={})
                out[i] = QuantizedModel(compressed_data=data, original_dimensions=(n, n), parameter_count=d,
                                        compression_quality=quality, hierarchical_indices=idx_h[k].copy(), metadata=md)
                if mm_h[k, 1] != mm_h[k, 0] and (last_state is None or i > last_state[0]):
                    last_state = (i, mm_h[k, 0], mm_h[k, 1])
                if pre_h is not None:
                    levels = [PrecomputedLevel(g, s_, c, pre_h[k, o:o + c].copy(), _square_coordinates(n, g, s_))
                              for (g, s_, c, o) in layout]
                    tot = sum(lv.averages.nbytes + len(lv.square_coordinates) * 16 for lv in levels)
                    hq.precomputed_indexer._index_cache[names[i]] = PrecomputedIndex(names[i], (n, n), levels, 0.0,
                                                                                     tot)
                    if verbose:
                        print(f"Pre-computing {len(levels)} granularity levels for {names[i]}...")
    for i in range(stop):
        if out[i] is None:  # non-float32 vectors: the per-model drop-in path (registers itself)
            out[i] = hq.quantize(sets[i], names[i], descs[i], validate=False)
            continue
        hq._model_registry.append(out[i])
    if last_state is not None:
        pipe.compressor._norm_min = np.float32(last_state[1])
        pipe.compressor._norm_max = np.float32(last_state[2])
    if stop_exc is not None:
        stop_exc.hq_quantized = out  # models quantized and registered before the failing one
        raise stop_exc
    return out


class BatchQuantizer:
    """api.py:567-650 drop-in: BatchQuantizer(config).quantize_batch / search_batch, batched on the GPU
    (one fused launch per vector length, one resident corpus per search batch)."""

    def __init__(self, config: Optional[SystemConfig] = None):
        self.quantizer = HilbertQuantizer(config)
        self.logger = logging.getLogger(__name__)

    def quantize_batch(self, parameter_sets, model_ids: Optional[List[str]] = None,
                       descriptions: Optional[List[str]] = None, parallel: bool = True) -> List[QuantizedModel]:
        if model_ids and len(model_ids) != len(parameter_sets):
            raise ValueError("Number of model IDs must match number of parameter sets")
        if descriptions and len(descriptions) != len(parameter_sets):
            raise ValueError("Number of descriptions must match number of parameter sets")
        return _ingest(self.quantizer, parameter_sets, model_ids, descriptions, parallel)

    def search_batch(self, query_sets, candidate_models: List[QuantizedModel],
                     max_results: int = 10) -> List[List[SearchResult]]:
        """api.py:621-650: quantizer.search per query (a failing query yields []).  With an explicit
        candidate pool the queries are quantized in one batch (registered in order, as search() does)
        and answered by one batched progressive scan; without one, the pool is the growing registry
        and the queries run one by one, exactly as the reference."""
        hq = self.quantizer
        if not candidate_models:
            out = []
            for q in query_sets:
                try:
                    out.append(hq.search(q, candidate_models, max_results))
                except Exception as e:
                    self.logger.error(f"Failed search: {e}")
                    out.append([])
            return out
        ok, models = [], []
        for i, q in enumerate(query_sets):
            q = np.array(q, dtype=np.float32) if isinstance(q, list) else q
            try:
                hq._validate_parameters(q)
                ok.append((i, q))
            except Exception as e:
                self.logger.error(f"Failed search {i + 1}: {e}")
        results: List[List[SearchResult]] = [[] for _ in query_sets]
        # quantize the valid queries in batches; a query whose quantize fails (dimension / efficiency
        # check) yields [] and the queries after it continue, as the reference's per-query loop does
        done = []  # (query position, QuantizedModel)
        pending = ok
        while pending:
            try:
                models = _ingest(hq, [q for _, q in pending], [f"model_{int(time.time())}" for _ in pending], None,
                                 True, validate=False)
                done.extend((i, m) for (i, _), m in zip(pending, models))
                pending = []
            except Exception as e:
                part = getattr(e, "hq_quantized", None)
                if part is None:  # not a per-query failure: answer the rest one query at a time
                    for i, q in pending:
                        try:
                            results[i] = hq.search(q, candidate_models, max_results)
                        except Exception as e2:
                            self.logger.error(f"Failed search {i + 1}: {e2}")
                    pending = []
                    break
                done.extend((i, m) for (i, _), m in zip(pending, part))
                self.logger.error(f"Failed search {pending[len(part)][0] + 1}: {e}")
                pending = pending[len(part) + 1:]
        if not done:
            return results
        found = hq.search_engine.progressive_search_batch([m.hierarchical_indices for _, m in done],
                                                          candidate_models, max_results)
        thr = hq.similarity_threshold
        for (i, _), res in zip(done, found):
            results[i] = [r for r in res if r.similarity_score >= thr]
        return results

    def reconstruct_batch(self, quantized_models: List[QuantizedModel]) -> List[np.ndarray]:
        """Batched reconstruct (HilbertQuantizer.reconstruct_many)."""
        return self.quantizer.reconstruct_many(quantized_models)

    def quantize_device(self, parameters, index_space_size: Optional[int] = None):
        """f32 [N, d] -> (frames u8 [N, n+1, n], indices f64 [N, L], minmax f32 [N, 2]) on the GPU."""
        return quantize_batch(parameters, self.quantizer.min_efficiency_ratio, index_space_size)

    @staticmethod
    def build_corpus(indices, id_base: int = 0) -> IndexCorpus:
        return IndexCorpus(indices, id_base)
