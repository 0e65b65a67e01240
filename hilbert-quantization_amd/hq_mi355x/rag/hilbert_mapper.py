"""RAG Hilbert mapper (rag/embedding_generation/hilbert_mapper.py:9-229): the same GPU maps as
hq_mi355x.core.HilbertCurveMapper with the RAG module's ValueError contract and messages."""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

from ..core.hilbert_mapper import HilbertCurveMapper
from ..exceptions import HilbertQuantizationError


class HilbertCurveMapperImpl:
    def __init__(self, config=None):
        self.config = config
        self._core = HilbertCurveMapper()

    def map_to_2d(self, embeddings, dimensions: Tuple[int, int]):
        width, height = dimensions
        if width <= 0 or height <= 0:
            raise ValueError(f"Dimensions must be positive, got {width}x{height}")
        if width != height:
            raise ValueError(f"Hilbert curve requires square dimensions, got {width}x{height}")
        if (width & (width - 1)) != 0:
            raise ValueError(f"Dimension must be a power of 2, got {width}")
        if len(embeddings) > width * height:
            raise ValueError(f"Too many embedding values ({len(embeddings)}) for dimensions {width}x{height} "
                             f"({width * height} cells)")
        return self._core.map_to_2d(embeddings, dimensions)

    def map_from_2d(self, image):
        if len(image.shape) != 2:
            raise ValueError(f"Input must be 2D array, got {len(image.shape)}D")
        height, width = image.shape
        if width != height:
            raise ValueError(f"Hilbert curve requires square dimensions, got {width}x{height}")
        if width <= 0 or (width & (width - 1)) != 0:
            raise ValueError(f"Dimension must be a power of 2, got {width}")
        return self._core.map_from_2d(image)

    def generate_hilbert_coordinates(self, n: int) -> List[Tuple[int, int]]:
        try:
            return self._core.generate_hilbert_coordinates(n)
        except HilbertQuantizationError as e:
            raise ValueError(str(e))

    def _hilbert_index_to_xy(self, index: int, n: int) -> Tuple[int, int]:
        return self._core._hilbert_index_to_xy(index, n)

    def _xy_to_hilbert_index(self, x: int, y: int, n: int) -> int:
        return self._core._xy_to_hilbert_index(x, y, n)

    def _rotate(self, n, x, y, rx, ry):
        return self._core._rotate(n, x, y, rx, ry)
