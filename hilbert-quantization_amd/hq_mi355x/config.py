"""Configuration dataclasses of the reference (hilbert_quantization/config.py:14-230), reduced to
the fields the hot path and HilbertQuantizer read, with the same defaults and validation messages.
The reference's ConfigurationManager / file persistence are out of scope."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Tuple


class Constants:
    VALID_DIMENSIONS = [4, 16, 64, 256, 1024, 4096, 16384]
    DEFAULT_PADDING_VALUE = 0.0
    INDEX_ALLOCATION_RATIOS = [0.5, 0.25, 0.125, 0.0625, 0.03125]
    MIN_EFFICIENCY_RATIO = 0.5
    DEFAULT_COMPRESSION_QUALITY = 0.8
    DEFAULT_MAX_SEARCH_RESULTS = 10
    DEFAULT_SIMILARITY_THRESHOLD = 0.1


@dataclass
class QuantizationConfig:
    auto_select_dimensions: bool = True
    target_dimensions: Optional[Tuple[int, int]] = None
    padding_value: float = Constants.DEFAULT_PADDING_VALUE
    min_efficiency_ratio: float = Constants.MIN_EFFICIENCY_RATIO
    use_streaming_optimization: bool = False
    strict_validation: bool = False

    def __post_init__(self):
        if not 0 <= self.min_efficiency_ratio <= 1:
            raise ValueError("Minimum efficiency ratio must be between 0 and 1")


@dataclass
class CompressionConfig:
    quality: float = Constants.DEFAULT_COMPRESSION_QUALITY
    preserve_index_row: bool = True
    validate_reconstruction: bool = True
    max_reconstruction_error: float = 0.01

    def __post_init__(self):
        if not 0 <= self.quality <= 1:
            raise ValueError("Compression quality must be between 0 and 1")
        if self.max_reconstruction_error < 0:
            raise ValueError("Maximum reconstruction error must be non-negative")


@dataclass
class SearchConfig:
    max_results: int = Constants.DEFAULT_MAX_SEARCH_RESULTS
    similarity_threshold: float = Constants.DEFAULT_SIMILARITY_THRESHOLD
    max_candidates_per_level: int = 1000

    def __post_init__(self):
        if self.max_results <= 0:
            raise ValueError("Maximum results must be positive")
        if not 0 <= self.similarity_threshold <= 1:
            raise ValueError("Similarity threshold must be between 0 and 1")
        if self.max_candidates_per_level <= 0:
            raise ValueError("Maximum candidates per level must be positive")


@dataclass
class SystemConfig:
    quantization: QuantizationConfig = field(default_factory=QuantizationConfig)
    compression: CompressionConfig = field(default_factory=CompressionConfig)
    search: SearchConfig = field(default_factory=SearchConfig)
    enable_logging: bool = True
    log_level: str = "INFO"


def create_default_config() -> SystemConfig:
    return SystemConfig()
