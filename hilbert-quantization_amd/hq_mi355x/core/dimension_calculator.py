"""Grid-size selection, host-side shape logic.

Same contract as the reference's core/dimension_calculator.py:36-128: n = sqrt of the first entry of
VALID_DIMENSIONS >= d (x4 beyond 16384); calculate_padding_strategy raises
ValueError("Efficiency ratio {r:.3f} is below minimum {m}") when d / n^2 < min_efficiency_ratio.
"""
from __future__ import annotations

import math
from typing import List, Tuple

from ..models import PaddingConfig
from .._compat import bases as _bases

VALID_DIMENSIONS = [4, 16, 64, 256, 1024, 4096, 16384]
MIN_EFFICIENCY_RATIO = 0.5
DEFAULT_PADDING_VALUE = 0.0


def _power_of_4_at_least(count: int) -> int:
    if count <= 0:
        return 4
    for size in VALID_DIMENSIONS:
        if size >= count:
            return size
    size = VALID_DIMENSIONS[-1]
    while size < count:
        size *= 4
    return size


def _optimal_side(count: int) -> int:
    return int(math.isqrt(_power_of_4_at_least(count)))


class PowerOf4DimensionCalculator(*_bases("interfaces", "DimensionCalculator")):
    def __init__(self, min_efficiency_ratio: float = MIN_EFFICIENCY_RATIO):
        self.min_efficiency_ratio = min_efficiency_ratio

    def calculate_optimal_dimensions(self, param_count: int) -> Tuple[int, int]:
        if param_count <= 0:
            raise ValueError("Parameter count must be positive")
        side = _optimal_side(param_count)
        return (side, side)

    def calculate_padding_strategy(self, param_count: int, target_dims: Tuple[int, int]) -> PaddingConfig:
        w, h = target_dims
        cells = w * h
        if cells < param_count:
            raise ValueError(f"Target dimensions {target_dims} cannot accommodate {param_count} parameters")
        ratio = param_count / cells
        if ratio < self.min_efficiency_ratio:
            raise ValueError(f"Efficiency ratio {ratio:.3f} is below minimum {self.min_efficiency_ratio}")
        # row-major tail cells, last cell first (:105-128) — informational only
        tail = [((cells - 1 - i) % w, (cells - 1 - i) // w) for i in range(cells - param_count)]
        return PaddingConfig(target_dimensions=target_dims, padding_value=DEFAULT_PADDING_VALUE,
                             padding_positions=tail, efficiency_ratio=ratio)

    def _find_nearest_power_of_4(self, value: int) -> int:
        return _power_of_4_at_least(value)

    def get_efficiency_metrics(self, param_count: int, dimensions: Tuple[int, int]) -> dict:
        w, h = dimensions
        cells = w * h
        return {"total_space": cells, "used_space": param_count, "wasted_space": cells - param_count,
                "efficiency_ratio": param_count / cells,
                "waste_percentage": (cells - param_count) / cells * 100, "dimensions": dimensions}

    def find_optimal_embedding_dimensions(self, embedding_size: int) -> Tuple[int, int]:
        if embedding_size <= 0:
            raise ValueError("Embedding size must be positive")
        return self.calculate_optimal_dimensions(embedding_size)


def validate_power_of_4(value: int) -> bool:
    if value <= 0:
        return False
    while value > 1:
        if value % 4:
            return False
        value //= 4
    return True
