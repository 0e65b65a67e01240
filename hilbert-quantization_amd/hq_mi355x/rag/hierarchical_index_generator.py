"""RAG multi-row hierarchical index on MI355X.

Drop-in for rag/embedding_generation/hierarchical_index_generator.py:14-627: granularity selection
is host-side shape logic (:23-101); the section means (np.mean in NumPy's pairwise order, visited
in the generator's Hilbert order including the hard-coded n=2 list of :302-303) run in
hq_index_rag_f32 / hq_block_means_f32."""
from __future__ import annotations

import math
from typing import Dict, List, Tuple

import numpy as np

from .. import kernels as K
from .._dev import is_tensor, to_dev, to_np


class HierarchicalIndexGenerator:
    def __init__(self, config=None):
        self.config = config or {}
        self.min_granularity = self.config.get("min_granularity", 2)
        self.max_index_rows = self.config.get("max_index_rows", 8)

    @staticmethod
    def _nearest_power_of_2(n: int) -> int:
        if n <= 0:
            return 1
        p = 1
        while p * 2 <= n:
            p *= 2
        return p

    def calculate_optimal_granularity(self, image_dimensions: Tuple[int, int]) -> Dict[str, object]:
        width, height = image_dimensions
        g = self._nearest_power_of_2(max(self.min_granularity, int(math.sqrt(width))))
        levels = []
        while g >= self.min_granularity and len(levels) < self.max_index_rows:
            levels.append(g)
            g //= 2
        return {"finest_granularity": levels[0] if levels else 0, "granularity_levels": levels,
                "index_rows_needed": len(levels), "total_image_height": height + len(levels),
                "original_dimensions": image_dimensions,
                "section_sizes": [(width // l, height // l) for l in levels]}

    def allocate_index_space(self, image_dimensions: Tuple[int, int]) -> Dict[str, object]:
        info = self.calculate_optimal_granularity(image_dimensions)
        width, height = image_dimensions
        rows = info["index_rows_needed"]
        return {"enhanced_dimensions": (width, height + rows),
                "index_row_positions": [height + i for i in range(rows)], "granularity_info": info}

    def _default_config(self) -> bool:
        return self.min_granularity == 2 and self.max_index_rows == 8

    def generate_multi_level_indices(self, embedding_image):
        if embedding_image.ndim != 2:
            raise ValueError("Embedding image must be 2D")
        h, w = embedding_image.shape
        img = embedding_image if is_tensor(embedding_image) else np.asarray(embedding_image)
        square = h == w and w > 0 and (w & (w - 1)) == 0
        if self._default_config() and square and str(img.dtype).endswith("float32"):
            out = K.index_rag(to_dev(img))
            return out if is_tensor(embedding_image) else to_np(out)
        # general shapes / configs: one block-mean launch per granularity row
        levels = self.calculate_optimal_granularity((w, h))["granularity_levels"]
        enh = np.zeros((h + len(levels), w), dtype=np.asarray(img).dtype)
        enh[:h] = to_np(img) if is_tensor(img) else img
        for i, g in enumerate(levels):
            row = self._calculate_hilbert_order_averages(enh[:h], g)
            k = min(len(row), w)
            enh[h + i, :k] = row[:k]
        return enh

    def create_progressive_granularity_levels(self, embedding_image) -> List[np.ndarray]:
        if embedding_image.ndim != 2:
            raise ValueError("Embedding image must be 2D")
        h, w = embedding_image.shape
        levels = self.calculate_optimal_granularity((w, h))["granularity_levels"]
        return [self._calculate_hilbert_order_averages(embedding_image, g) for g in levels]

    def _calculate_hilbert_order_averages(self, image, granularity: int) -> np.ndarray:
        img = np.asarray(image)
        h, w = img.shape
        if h != w or img.dtype not in (np.float32, np.float64):
            raise ValueError("GPU block means need a square float32/float64 image")
        return to_np(K.block_means(to_dev(img), int(granularity), 1))

    def embed_multi_level_indices(self, image, index_rows: List[np.ndarray]):
        if image.ndim != 2:
            raise ValueError("Image must be 2D")
        if not index_rows:
            return image.copy()
        h, w = image.shape
        enh = np.zeros((h + len(index_rows), w), dtype=image.dtype)
        enh[:h] = image
        for i, row in enumerate(index_rows):
            k = min(len(row), w)
            enh[h + i, :k] = np.asarray(row)[:k]
        return enh

    def generate_batch(self, images):
        """[N, n, n] f32 device images -> [N, n + R, n] enhanced images."""
        return K.index_rag(to_dev(images))
