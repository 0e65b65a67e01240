"""High-level API (reference hilbert_quantization/api.py:27-649) on the MI355X components.

HilbertQuantizer keeps quantize / reconstruct / search and the model registry with the reference's
exception wrapping (QuantizationError / ReconstructionError / SearchError / ValidationError).  The
search uses ProgressiveSimilaritySearchEngine(threshold, max_candidates_per_level = 2 * max_results)
as the reference does (api.py:93-101) and filters results >= threshold (:284-287).
BatchQuantizer adds the batched device path (one fused kernel for N embeddings).
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
from .exceptions import QuantizationError, ReconstructionError, SearchError, ValidationError
from .models import QuantizedModel, SearchResult


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

    def reconstruct(self, quantized_model: QuantizedModel, validate: bool = True) -> np.ndarray:
        try:
            return self.quantization_pipeline.reconstruct_parameters(quantized_model)
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


class BatchQuantizer:
    """Batched device path: one fused launch per batch, indices kept resident for search."""

    def __init__(self, min_efficiency_ratio: float = 0.5):
        self.min_efficiency_ratio = min_efficiency_ratio

    def quantize_batch(self, parameters, index_space_size: Optional[int] = None):
        """f32 [N, d] -> (frames u8 [N, n+1, n], indices f64 [N, L], minmax f32 [N, 2]) on the GPU."""
        return quantize_batch(parameters, self.min_efficiency_ratio, index_space_size)

    @staticmethod
    def build_corpus(indices, id_base: int = 0) -> IndexCorpus:
        return IndexCorpus(indices, id_base)
