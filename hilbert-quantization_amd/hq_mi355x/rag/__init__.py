"""RAG-side components (hilbert_quantization.rag.*) backed by libhq_mi355x."""
from .hilbert_mapper import HilbertCurveMapperImpl
from .hierarchical_index_generator import HierarchicalIndexGenerator
from .similarity import (calculate_embedding_cosine_similarity, compare_single_level_indices,
                         compare_multi_level_indices, calculate_granularity_weights,
                         calculate_spatial_locality_similarity, cosine_scores_batch)

__all__ = ["HilbertCurveMapperImpl", "HierarchicalIndexGenerator", "calculate_embedding_cosine_similarity",
           "compare_single_level_indices", "compare_multi_level_indices", "calculate_granularity_weights",
           "calculate_spatial_locality_similarity", "cosine_scores_batch"]
