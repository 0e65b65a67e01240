"""Exception hierarchy of the drop-in (same class names as the reference's exceptions.py:1-77 so
callers' `except` clauses and the reference tests' `pytest.raises(..., match=...)` keep working).
When the reference package is importable, every class also subclasses the reference's exception of
the same name (_compat.bases), so a reference caller's `except` clause catches it."""
from ._compat import bases as _b


class HilbertQuantizationError(*_b("exceptions", "HilbertQuantizationError", Exception)):
    pass


class DimensionCalculationError(*_b("exceptions", "DimensionCalculationError", HilbertQuantizationError)):
    pass


class HilbertMappingError(*_b("exceptions", "HilbertMappingError", HilbertQuantizationError)):
    pass


class IndexGenerationError(*_b("exceptions", "IndexGenerationError", HilbertQuantizationError)):
    pass


class CompressionError(*_b("exceptions", "CompressionError", HilbertQuantizationError)):
    pass


class SearchError(*_b("exceptions", "SearchError", HilbertQuantizationError)):
    pass


class ValidationError(*_b("exceptions", "ValidationError", HilbertQuantizationError)):
    pass


class ConfigurationError(*_b("exceptions", "ConfigurationError", HilbertQuantizationError)):
    pass


class QuantizationError(*_b("exceptions", "QuantizationError", HilbertQuantizationError)):
    pass


class ReconstructionError(*_b("exceptions", "ReconstructionError", HilbertQuantizationError)):
    pass
