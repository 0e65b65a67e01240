"""Reference-shaped core components (hilbert_quantization.core.*) backed by libhq_mi355x."""
from .dimension_calculator import PowerOf4DimensionCalculator
from .hilbert_mapper import HilbertCurveMapper
from .streaming_index_builder import StreamingHilbertIndexGenerator
from .index_generator import HierarchicalIndexGeneratorImpl
from .compressor import MPEGAICompressorImpl
from .search_engine import ProgressiveSimilaritySearchEngine, LevelConfig, IndexCorpus
from .pipeline import QuantizationPipeline, quantize_batch
from .precomputed_hilbert_index import (PrecomputedHilbertIndexer, PrecomputedSimilaritySearchEngine,
                                        PrecomputedIndex, PrecomputedLevel)

__all__ = ["PowerOf4DimensionCalculator", "HilbertCurveMapper", "StreamingHilbertIndexGenerator",
           "HierarchicalIndexGeneratorImpl", "MPEGAICompressorImpl", "ProgressiveSimilaritySearchEngine",
           "LevelConfig", "IndexCorpus", "QuantizationPipeline", "quantize_batch", "PrecomputedHilbertIndexer",
           "PrecomputedSimilaritySearchEngine", "PrecomputedIndex", "PrecomputedLevel"]
