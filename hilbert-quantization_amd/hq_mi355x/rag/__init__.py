"""RAG-side components (hilbert_quantization.rag.*) backed by libhq_mi355x."""
from .hilbert_mapper import HilbertCurveMapperImpl
from .hierarchical_index_generator import HierarchicalIndexGenerator
from .similarity import (apply_progressive_threshold, calculate_embedding_cosine_similarity,
                         calculate_granularity_weights, calculate_spatial_locality_similarity,
                         compare_multi_level_indices, compare_single_level_indices, cosine_scores_batch,
                         detect_original_embedding_height, extract_original_embedding, progressive_threshold,
                         progressive_threshold_batch, spatial_locality_scores)

__all__ = ["HilbertCurveMapperImpl", "HierarchicalIndexGenerator", "apply_progressive_threshold",
           "calculate_embedding_cosine_similarity", "calculate_granularity_weights",
           "calculate_spatial_locality_similarity", "compare_multi_level_indices", "compare_single_level_indices",
           "cosine_scores_batch", "detect_original_embedding_height", "extract_original_embedding",
           "progressive_threshold", "progressive_threshold_batch", "spatial_locality_scores"]
