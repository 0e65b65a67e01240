"""Binding to the reference's own types.

When the reference package `hilbert_quantization` is importable in the same process, the drop-in's
classes join its type hierarchy instead of standing beside it:
* the exceptions subclass the reference's exception of the same name (exceptions.py:6-77), so a
  reference caller's `except QuantizationError` catches this package's errors;
* the GPU components subclass the reference ABCs they implement (interfaces.py:12-225:
  DimensionCalculator, HilbertCurveMapper, HierarchicalIndexGenerator, MPEGAICompressor,
  SimilaritySearchEngine), so `isinstance` checks and constructor injection accept them;
* the data model IS the reference's (models.py:11-80 QuantizedModel, SearchResult, ModelMetadata,
  PaddingConfig): results carry the reference's own dataclasses.
Without the reference (the GPU box, a plain install) the package uses its own field-for-field copies.
Nothing here imports the reference unless it is installed; a reference that fails to import (e.g. its
OpenCV dependency missing) counts as absent.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
from typing import Optional, Tuple

_cache = {}


def reference_module(name: str):
    """hilbert_quantization.<name>, or None when the reference package is not importable (or binding is
    switched off with HQ_NO_REFERENCE_BINDING=1)."""
    if name in _cache:
        return _cache[name]
    mod = None
    if os.environ.get("HQ_NO_REFERENCE_BINDING") != "1":
        try:
            if importlib.util.find_spec("hilbert_quantization") is not None:
                mod = importlib.import_module(f"hilbert_quantization.{name}")
        except Exception:
            mod = None
    _cache[name] = mod
    return mod


def ref_class(module: str, name: str) -> Optional[type]:
    m = reference_module(module)
    c = getattr(m, name, None) if m is not None else None
    return c if isinstance(c, type) else None


def bases(module: str, name: str, *own) -> Tuple[type, ...]:
    """Base classes for a drop-in class: its own bases, then the reference class of that name if any."""
    c = ref_class(module, name)
    if c is None:
        return tuple(own)
    # own bases the reference class already derives from (e.g. Exception) are left to it (a valid MRO)
    return tuple(b for b in own if not issubclass(c, b)) + (c,)
