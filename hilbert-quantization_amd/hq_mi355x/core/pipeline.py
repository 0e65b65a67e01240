"""Quantization pipeline on MI355X (SURVEY.md §8a rows S1, P1, M5, I1, I3, Q1 fused).

`quantize_batch` is the batched north-star path: f32 [N, d] parameters -> uint8 frames
[N, n+1, n], float64 streaming indices [N, L] and per-frame (min, max), in ONE kernel
(hq_map_index_quantize) — the component sequence of the reference's
QuantizationPipeline.quantize_model (core/pipeline.py:97-146) without the JPEG codec.
`QuantizationPipeline` keeps the reference's constructor injection and quantize_model /
reconstruct_parameters surface for per-model use.
"""
from __future__ import annotations

import time
from typing import Any, Dict, Optional

import numpy as np

from .. import kernels as K
from .._dev import to_dev, to_np, torch
from ..exceptions import HilbertQuantizationError
from ..models import ModelMetadata, QuantizedModel
from .compressor import MPEGAICompressorImpl
from .dimension_calculator import PowerOf4DimensionCalculator
from .hilbert_mapper import HilbertCurveMapper
from .index_generator import HierarchicalIndexGeneratorImpl, QuantizationConfig


def quantize_batch(parameters, min_efficiency_ratio: float = 0.5, index_space_size: Optional[int] = None,
                   out=None):
    """Fused map + streaming index + embed + uint8 quantize for a batch of equal-length vectors.

    parameters: f32 [N, d] (NumPy or device tensor).  The grid side n follows
    PowerOf4DimensionCalculator and its efficiency check (raises ValueError exactly like the
    reference for d / n^2 < min_efficiency_ratio).  Returns device tensors
    (frames u8 [N, n+1, n], indices f64 [N, L], minmax f32 [N, 2]) with L = n by default
    (core/pipeline.py:112 `index_space_size = dimensions[0]`)."""
    t = torch()
    x = to_dev(parameters)
    if x.dim() == 1:
        x = x.view(1, -1)
    if x.dtype != t.float32:
        raise TypeError("quantize_batch takes float32 parameters (the reference's embedding dtype)")
    d = int(x.shape[1])
    calc = PowerOf4DimensionCalculator(min_efficiency_ratio)
    dims = calc.calculate_optimal_dimensions(d)
    calc.calculate_padding_strategy(d, dims)
    n = dims[0]
    L = n if index_space_size is None else int(index_space_size)
    return K.map_index_quantize(x, n, L, out=out)


class QuantizationPipeline:
    """core/pipeline.py:29 drop-in with GPU components injected by default."""

    def __init__(self, dimension_calculator=None, hilbert_mapper=None, index_generator=None, compressor=None,
                 compression_config=None, use_streaming_optimization: bool = True):
        self.dimension_calculator = dimension_calculator or PowerOf4DimensionCalculator()
        self.hilbert_mapper = hilbert_mapper or HilbertCurveMapper()
        if use_streaming_optimization and index_generator is None:
            self.index_generator = HierarchicalIndexGeneratorImpl(QuantizationConfig(use_streaming_optimization=True))
        else:
            self.index_generator = index_generator or HierarchicalIndexGeneratorImpl()
        self.compressor = compressor or MPEGAICompressorImpl(compression_config)
        self.compression_config = compression_config
        self.use_streaming_optimization = use_streaming_optimization

    def _pad_parameters(self, parameters, dimensions, padding_config=None):
        total = dimensions[0] * dimensions[1]
        p = np.asarray(parameters)
        if len(p) >= total:
            return p[:total]
        out = np.zeros(total, dtype=p.dtype)
        out[: len(p)] = p
        return out

    def quantize_model(self, parameters, model_name: str, compression_quality: float = 0.8,
                       model_architecture: Optional[str] = None,
                       additional_metadata: Optional[Dict[str, Any]] = None) -> QuantizedModel:
        try:
            dims = self.dimension_calculator.calculate_optimal_dimensions(len(parameters))
            pc = self.dimension_calculator.calculate_padding_strategy(len(parameters), dims)
            padded = self._pad_parameters(parameters, dims, pc)
            image = self.hilbert_mapper.map_to_2d(padded, dims)
            idx = self.index_generator.generate_optimized_indices(image, dims[0])
            enhanced = self.index_generator.embed_indices_in_image(image, idx)
            data = self.compressor.compress(enhanced, compression_quality)
            size = np.asarray(parameters).nbytes
            md = ModelMetadata(model_name=model_name, original_size_bytes=size, compressed_size_bytes=len(data),
                               compression_ratio=size / len(data) if data else 0.0,
                               quantization_timestamp=time.strftime("%Y-%m-%d %H:%M:%S"),
                               model_architecture=model_architecture, additional_info=additional_metadata or {})
            return QuantizedModel(compressed_data=data, original_dimensions=dims, parameter_count=len(parameters),
                                  compression_quality=compression_quality, hierarchical_indices=idx, metadata=md)
        except Exception as e:
            raise HilbertQuantizationError(f"Failed to quantize model '{model_name}': {e}")

    def _get_2d_representation(self, parameters):
        """core/pipeline.py:298-323: pad + Hilbert map (the image the pre-computed index is built on)."""
        try:
            dims = self.dimension_calculator.calculate_optimal_dimensions(len(parameters))
            pc = self.dimension_calculator.calculate_padding_strategy(len(parameters), dims)
            return self.hilbert_mapper.map_to_2d(self._pad_parameters(parameters, dims, pc), dims)
        except Exception as e:
            raise HilbertQuantizationError(f"Failed to get 2D representation: {e}")

    def reconstruct_parameters(self, quantized_model: QuantizedModel):
        try:
            enhanced = self.compressor.decompress(quantized_model.compressed_data)
            image, _ = self.index_generator.extract_indices_from_image(enhanced)
            flat = self.hilbert_mapper.map_from_2d(image)
            out = flat[: quantized_model.parameter_count]
            if len(out) != quantized_model.parameter_count:
                raise HilbertQuantizationError(
                    f"Reconstructed parameter count {len(out)} doesn't match original {quantized_model.parameter_count}")
            return out
        except Exception as e:
            raise HilbertQuantizationError(f"Failed to reconstruct parameters: {e}")


def reconstruct_batch(models, compressor: MPEGAICompressorImpl, workers: int = 16):
    """Batched QuantizationPipeline.reconstruct_parameters (core/pipeline.py:183-235) for
    many QuantizedModels: the JPEG payloads decode on a host thread pool (the codec), then per frame shape
    ONE de-normalise launch (hq_dequantize_u8, with the compressor instance's last (min, max) for every
    model, exactly as the per-model path reads that shared state) and ONE inverse-Hilbert gather
    (hq_map_from_2d) of the image rows above the index row; each model's vector is truncated to its
    parameter count.  Returns float32 NumPy vectors in model order; the errors are the per-model path's
    (HilbertQuantizationError wrapping the decompress / shape failure of the first failing model)."""
    import concurrent.futures as cf
    from .compressor import check_payload, decode_jpeg
    t = torch()
    models = list(models)
    out = [None] * len(models)

    def decode(i):
        m = models[i]
        try:
            check_payload(m.compressed_data)
            try:
                return decode_jpeg(m.compressed_data)
            except Exception as e:
                raise RuntimeError(f"Failed to decompress image: {e}")
        except Exception as e:
            raise HilbertQuantizationError(f"Failed to reconstruct parameters: {e}")

    with cf.ThreadPoolExecutor(max_workers=max(1, min(workers, len(models) or 1))) as pool:
        frames = list(pool.map(decode, range(len(models))))
    mm = compressor._state_minmax()
    groups = {}
    for i, f in enumerate(frames):
        groups.setdefault(f.shape, []).append(i)
    for shape, members in groups.items():
        u8 = to_dev(np.stack([frames[i] for i in members]))
        enh = K.dequantize_u8(u8, to_dev(np.repeat(mm[None], len(members), 0)), HilbertQuantizationError)
        r, c = shape
        if r < 2 or r - 1 != c or (c & (c - 1)) != 0:  # not an (n + 1) x n enhanced frame: per-model path
            for i in members:
                out[i] = None
            continue
        flat = to_np(K.map_from_2d(enh[:, :-1, :].contiguous(), None, HilbertQuantizationError))
        for k, i in enumerate(members):
            v = flat[k, : models[i].parameter_count]
            if len(v) != models[i].parameter_count:
                raise HilbertQuantizationError(
                    f"Failed to reconstruct parameters: Reconstructed parameter count {len(v)} doesn't match "
                    f"original {models[i].parameter_count}")
            out[i] = v.copy()
    return out
