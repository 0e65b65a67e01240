"""hq_mi355x — MI355X-native hot path of hilbert_quantization (Hilbert map, hierarchical indices,
uint8 frame quantize, hierarchical-index similarity scan).

All arithmetic runs in hand-written HIP kernels for gfx950 (libhq_mi355x.so, C-ABI in
include/hq_mi355x.h); torch tensors are used only as HBM buffers.  The module layout mirrors the
reference package (`core`, `rag`, `api`, `models`, `exceptions`) so it drops in behind
hilbert_quantization.api and .rag.
"""
from .exceptions import (HilbertQuantizationError, QuantizationError, ReconstructionError, SearchError,
                         ValidationError, CompressionError)
from .models import QuantizedModel, SearchResult, ModelMetadata, PaddingConfig
from ._lib import NativeLibraryError
from . import kernels

__version__ = "0.1.0"


def library_path() -> str:
    from ._lib import LIB_PATH
    return LIB_PATH


def __getattr__(name):
    # lazy: importing the package must not require a GPU (CPU-side tests load only the library)
    if name in ("core", "rag", "api", "distributed"):
        import importlib
        return importlib.import_module(f".{name}", __name__)
    if name in ("HilbertQuantizer", "BatchQuantizer"):
        from . import api
        return getattr(api, name)
    raise AttributeError(name)
