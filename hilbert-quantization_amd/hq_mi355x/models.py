"""Data model of the drop-in: field-for-field the reference's models.py:10-80 dataclasses
(QuantizedModel, SearchResult, ModelMetadata, PaddingConfig) with the same validation rules, so
objects flow unchanged between the reference's orchestration code and this package."""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple

import numpy as np


@dataclass
class ModelMetadata:
    model_name: str
    original_size_bytes: int
    compressed_size_bytes: int
    compression_ratio: float
    quantization_timestamp: str
    model_architecture: Optional[str] = None
    additional_info: Optional[Dict[str, Any]] = None
    compression_metrics: Optional[Any] = None


@dataclass
class PaddingConfig:
    target_dimensions: Tuple[int, int]
    padding_value: float
    padding_positions: List[Tuple[int, int]]
    efficiency_ratio: float

    def __post_init__(self):
        if not 0 <= self.efficiency_ratio <= 1:
            raise ValueError("Efficiency ratio must be between 0 and 1")
        if len(self.target_dimensions) != 2:
            raise ValueError("Target dimensions must be a 2-tuple")


@dataclass
class SearchResult:
    model: "QuantizedModel"
    similarity_score: float
    matching_indices: Dict[int, float]
    reconstruction_error: float

    def __post_init__(self):
        if not 0 <= self.similarity_score <= 1:
            raise ValueError("Similarity score must be between 0 and 1")
        if self.reconstruction_error < 0:
            raise ValueError("Reconstruction error must be non-negative")


@dataclass
class QuantizedModel:
    compressed_data: bytes
    original_dimensions: Tuple[int, int]
    parameter_count: int
    compression_quality: float
    hierarchical_indices: np.ndarray
    metadata: ModelMetadata

    @property
    def model_id(self) -> str:
        return self.metadata.model_name

    def __post_init__(self):
        if self.parameter_count <= 0:
            raise ValueError("Parameter count must be positive")
        if not 0 <= self.compression_quality <= 1:
            raise ValueError("Compression quality must be between 0 and 1")
        if len(self.original_dimensions) != 2:
            raise ValueError("Original dimensions must be a 2-tuple")
        if self.hierarchical_indices.ndim != 1:
            raise ValueError("Hierarchical indices must be 1-dimensional")


# With the reference package importable, the data model IS the reference's (same fields and validation):
# results and models then carry the reference's own dataclasses (_compat).
from ._compat import ref_class as _ref_class  # noqa: E402

for _name in ("ModelMetadata", "PaddingConfig", "SearchResult", "QuantizedModel"):
    _cls = _ref_class("models", _name)
    if _cls is not None:
        globals()[_name] = _cls
