"""HierarchicalIndexGeneratorImpl on MI355X.

Drop-in for the reference's core/index_generator.py:13-356: `use_streaming_optimization` selects the
streaming index (hq_index_streaming), otherwise the traditional block-mean/offset-sample index
(hq_index_traditional_f32, including the is_offset_sampling quirk of :329-332).  Allocation tables
are host-side integer logic, identical to :34-98.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np

from .. import kernels as K
from .._dev import is_tensor, to_dev, to_np
from .._compat import bases as _bases


class QuantizationConfig:
    """Minimal stand-in for the reference config object (config.py:40-110): only the switch read here."""

    def __init__(self, use_streaming_optimization: bool = False):
        self.use_streaming_optimization = use_streaming_optimization


def level_allocation(total_space: int) -> List[Tuple[int, int]]:
    """(grid, allocation) list, finest first, halving fractions, remainder to the finest grid."""
    if total_space <= 0:
        return []
    out: List[Tuple[int, int]] = []
    remaining = total_space
    cap = min(32, int(math.sqrt(total_space)))
    g = 1
    while g <= cap:
        g *= 2
    g = max(g // 2, 2)
    frac = 0.5
    while remaining > 0 and g >= 1:
        a = min(int(remaining * frac), g * g, remaining)
        if a > 0:
            out.append((g, a))
            remaining -= a
        g //= 2
        frac *= 0.5
        if frac < 0.01:
            break
    if remaining > 0 and out:
        out.append((out[0][0], remaining))
    return out


class HierarchicalIndexGeneratorImpl(*_bases("interfaces", "HierarchicalIndexGenerator")):
    def __init__(self, config: Optional[object] = None):
        self.config = config or QuantizationConfig()
        if getattr(self.config, "use_streaming_optimization", False):
            from .streaming_index_builder import StreamingHilbertIndexGenerator
            self._streaming_generator = StreamingHilbertIndexGenerator()
        else:
            self._streaming_generator = None

    def calculate_level_allocation(self, total_space: int) -> List[Tuple[int, int]]:
        return level_allocation(total_space)

    def calculate_spatial_averages(self, image, grid_size: int) -> List[float]:
        if image.size == 0 or grid_size <= 0:
            return []
        img = np.asarray(image)
        if img.dtype not in (np.float32, np.float64):
            img = img.astype(np.float64)
        return [float(v) for v in to_np(K.block_means(to_dev(img), int(grid_size), 0))]

    def calculate_offset_samples(self, image, section_size: int, available_space: int) -> List[float]:
        """Corner + centre pixels of row-major sections (pure pixel selection, :146-219)."""
        if image.size == 0 or section_size <= 0 or available_space <= 0:
            return []
        h, w = image.shape
        sy, sx = h // section_size, w // section_size
        if sy == 0 or sx == 0:
            picks = [(0, 0), (0, w - 1), (h - 1, 0), (h - 1, w - 1), (h // 2, w // 2)]
            return [float(image[r, c]) for r, c in picks][:available_space]
        nsec = min(available_space // 5, sy * sx)
        out: List[float] = []
        for k in range(nsec):
            r, c = divmod(k, sx)
            r0, r1 = r * section_size, min((r + 1) * section_size, h)
            c0, c1 = c * section_size, min((c + 1) * section_size, w)
            for (y, x) in ((r0, c0), (r0, c1 - 1), (r1 - 1, c0), (r1 - 1, c1 - 1), ((r0 + r1) // 2, (c0 + c1) // 2)):
                out.append(float(image[y, x]))
        return out[:available_space]

    def embed_indices_in_image(self, image, indices):
        """(n+1) x n: image rows plus one index row cast to the image dtype, zero filled (:221-253)."""
        if image.size == 0:
            return image
        h, w = image.shape
        enh = np.zeros((h + 1, w), dtype=image.dtype)
        enh[:h] = image
        k = min(len(indices), w)
        enh[h, :k] = np.asarray(indices)[:k]
        return enh

    def extract_indices_from_image(self, enhanced_image) -> Tuple[np.ndarray, np.ndarray]:
        if enhanced_image.size == 0:
            return enhanced_image, np.array([])
        if enhanced_image.shape[0] < 2:
            return enhanced_image, np.array([])
        row = enhanced_image[-1, :]
        nz = np.nonzero(row)[0]
        row = row[: nz[-1] + 1] if len(nz) else row[:1]
        return enhanced_image[:-1, :], row

    def generate_optimized_indices(self, image, index_space_size: int):
        if image.size == 0 or index_space_size <= 0:
            return np.array([])
        if self._streaming_generator is not None:
            return self._streaming_generator.generate_optimized_indices(image, index_space_size)
        return self._generate_traditional_indices(image, index_space_size)

    def _generate_traditional_indices(self, image, index_space_size: int):
        if is_tensor(image):
            return K.index_traditional(to_dev(image), int(index_space_size))
        img = np.asarray(image, dtype=np.float32)
        h, w = img.shape
        if h != w or (w & (w - 1)) != 0:
            raise ValueError(f"traditional index on the GPU needs a square power-of-2 image, got {w}x{h}")
        return to_np(K.index_traditional(to_dev(img), int(index_space_size)))

    def generate_batch(self, images, index_space_size: int):
        """[N, n, n] device images -> device indices (f64 streaming / f32 traditional)."""
        x = to_dev(images)
        if self._streaming_generator is not None:
            return K.index_streaming(x, int(index_space_size))
        return K.index_traditional(x, int(index_space_size))
