"""Streaming hierarchical index on MI355X.

Drop-in for StreamingHilbertIndexGenerator (reference core/streaming_index_builder.py:274-343): the
4-ary float64 mean tree over the Hilbert-ordered stream and the per-level strided sampling
(:154-243) run in the `hq_index_streaming` kernel (or fused into `hq_map_index_quantize`).
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

from .. import kernels as K
from .._dev import is_tensor, to_dev, to_np

MAX_LEVELS = 10


def level_sizes(stream_len: int, max_levels: int = MAX_LEVELS):
    """Values per level of the mean tree for a stream of `stream_len` values (:45-102)."""
    sizes = []
    s = stream_len
    while len(sizes) < max_levels and s > 0:
        sizes.append(s)
        s //= 4
    return sizes


class StreamingHilbertIndexGenerator:
    def __init__(self):
        from .hilbert_mapper import HilbertCurveMapper
        self.hilbert_mapper = HilbertCurveMapper()

    @staticmethod
    def _check(image):
        height, width = image.shape[-2], image.shape[-1]
        if width != height or width <= 0 or (width & (width - 1)) != 0:
            raise ValueError(f"Image must be square with power-of-2 dimensions, got {width}x{height}")

    def generate_optimized_indices(self, image, index_space_size: int):
        self._check(image)
        if index_space_size <= 0:
            return np.array([])
        if is_tensor(image):
            return K.index_streaming(to_dev(image), int(index_space_size))
        img = np.asarray(image)
        if img.dtype not in (np.float32, np.float64):
            img = img.astype(np.float64)
        return to_np(K.index_streaming(to_dev(img), int(index_space_size)))

    def generate_indices_during_mapping(self, parameters, dimensions: Tuple[int, int], index_space_size: int):
        """(image, indices, stats) like the reference (:287-313), both products from GPU kernels."""
        image = self.hilbert_mapper.map_to_2d(parameters, dimensions)
        d = len(parameters)
        if index_space_size <= 0:
            idx = np.array([])
        else:
            img = image if is_tensor(image) else np.asarray(image)
            if not is_tensor(img) and img.dtype not in (np.float32, np.float64):
                img = img.astype(np.float64)
            idx = K.index_streaming(to_dev(img), int(index_space_size), stream_len=d)
            if not is_tensor(image):
                idx = to_np(idx)
        sizes = level_sizes(d)
        stats = {"total_values_processed": int(d), "levels_used": len(sizes),
                 "indices_per_level": {i: s for i, s in enumerate(sizes)}}
        return image, idx, stats

    def generate_batch(self, images, index_space_size: int):
        """[N, n, n] device images -> f64 [N, L] device indices."""
        x = to_dev(images)
        self._check(x)
        return K.index_streaming(x, int(index_space_size))
