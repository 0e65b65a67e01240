"""MPEGAICompressorImpl on MI355X: the uint8 normalise stage.

`_normalize_for_compression` / `_denormalize_from_compression` keep the reference's instance-state
semantics (core/compressor.py:256-303): a non-constant image stores (min, max) on the instance, a
constant image returns 128s and leaves the state untouched, and de-normalising without state is
u8 / 255.  The arithmetic runs in hq_quantize_u8 / hq_dequantize_u8.  The JPEG ("MPEG-AI") codec
after it is outside the hot path; `compress`/`decompress` wrap PIL on the host
exactly where the reference does so the pipeline stays usable end to end.
"""
from __future__ import annotations

import io
from typing import Optional

import numpy as np

from .. import kernels as K
from .._dev import to_dev, to_np
from ..exceptions import CompressionError
from .._compat import bases as _bases


def encode_jpeg(u8: np.ndarray, quality: float) -> bytes:
    """The reference's JPEG stage for an already normalised uint8 frame (core/compressor.py:71-80):
    PIL 'L' image, quality max(1, min(95, int(q * 95))), optimize=True.  Host codec;
    the same frame bytes give the same JPEG bytes as the per-model path."""
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(u8, "L").save(buf, format="JPEG", quality=max(1, min(95, int(quality * 95))), optimize=True)
    return buf.getvalue()


def check_payload(compressed_data) -> None:
    """core/compressor.py:121-124 argument checks of decompress."""
    if not isinstance(compressed_data, bytes):
        raise ValueError("Compressed data must be bytes")
    if len(compressed_data) == 0:
        raise ValueError("Compressed data cannot be empty")


def decode_jpeg(compressed_data: bytes) -> np.ndarray:
    """Host JPEG decode of one payload -> uint8 frame (the reference's np.array(Image.open(...)) values)."""
    from PIL import Image
    return np.array(Image.open(io.BytesIO(compressed_data)), dtype=np.uint8)


class MPEGAICompressorImpl(*_bases("interfaces", "MPEGAICompressor")):
    def __init__(self, config: Optional[object] = None):
        self.config = config
        self._last_compression_metrics = None

    def _normalize_for_compression(self, image):
        img = np.asarray(image)
        if img.dtype != np.float32:
            raise CompressionError(f"GPU normalise implements the float32 frame path, got {img.dtype}")
        u8, mm = K.quantize_u8(to_dev(img), CompressionError)
        mm = to_np(mm)
        if mm[1] != mm[0]:
            self._norm_min = np.float32(mm[0])
            self._norm_max = np.float32(mm[1])
        return to_np(u8)

    def _denormalize_from_compression(self, image):
        u8 = np.asarray(image, dtype=np.uint8)
        mm = self._state_minmax()  # no state: (0, 1), and u8 / 255 * 1 + 0 == u8 / 255 exactly
        return to_np(K.dequantize_u8(to_dev(u8), to_dev(mm), CompressionError))

    def compress(self, image, quality: float) -> bytes:
        """core/compressor.py:43-103: validation, GPU normalise, then the host JPEG codec."""
        if not isinstance(image, np.ndarray):
            raise ValueError("Image must be a numpy array")
        if image.ndim != 2:
            raise ValueError("Image must be 2-dimensional")
        if not 0.0 <= quality <= 1.0:
            raise ValueError("Quality must be between 0.0 and 1.0")
        try:
            return encode_jpeg(self._normalize_for_compression(image), quality)
        except Exception as e:
            raise RuntimeError(f"Failed to compress image: {e}")

    def decompress(self, compressed_data: bytes):
        """core/compressor.py:106-148: host JPEG decode, then the GPU de-normalise with this instance's
        last (min, max)."""
        check_payload(compressed_data)
        try:
            return self._denormalize_from_compression(decode_jpeg(compressed_data))
        except Exception as e:
            raise RuntimeError(f"Failed to decompress image: {e}")

    def _state_minmax(self) -> np.ndarray:
        """(min, max) the de-normalise uses: the instance's last non-constant frame, else (0, 1) = u8 / 255."""
        if not hasattr(self, "_norm_min") or not hasattr(self, "_norm_max"):
            return np.array([0.0, 1.0], dtype=np.float32)
        return np.array([self._norm_min, self._norm_max], dtype=np.float32)

    def estimate_compression_ratio(self, original_size: int, compressed_size: int) -> float:
        if compressed_size <= 0:
            raise ValueError("Compressed size must be positive")
        return original_size / compressed_size
