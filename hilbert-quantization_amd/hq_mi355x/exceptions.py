"""Exception hierarchy of the drop-in (same class names as the reference's exceptions.py:1-77 so
callers' `except` clauses and the reference tests' `pytest.raises(..., match=...)` keep working)."""


class HilbertQuantizationError(Exception):
    pass


class DimensionCalculationError(HilbertQuantizationError):
    pass


class HilbertMappingError(HilbertQuantizationError):
    pass


class IndexGenerationError(HilbertQuantizationError):
    pass


class CompressionError(HilbertQuantizationError):
    pass


class SearchError(HilbertQuantizationError):
    pass


class ValidationError(HilbertQuantizationError):
    pass


class ConfigurationError(HilbertQuantizationError):
    pass


class QuantizationError(HilbertQuantizationError):
    pass


class ReconstructionError(HilbertQuantizationError):
    pass
