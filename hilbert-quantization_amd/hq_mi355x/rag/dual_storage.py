"""RAG dual-video storage loader: the reference's dual storage metadata
(rag/video_storage/dual_storage.py:51-143) into a device-resident frame corpus for the S7 scorer.

`load_dual_storage_metadata` reads `<storage_root>/metadata/dual_video_metadata.json` exactly as the
reference's `_load_existing_metadata` (:51-84): missing file -> empty state; the two counters first, then
frame by frame (a DocumentChunk and a VideoFrameMetadata per entry, hierarchical_indices left empty — the
reference loads them "separately if needed"); an exception stops the loop with the reference's printed
warning and keeps what was read before it.  The embedding frames themselves live in the storage's mp4
files (OpenCV codec, out of scope): `DualStorageCorpus` takes them decoded, in frame order, and keeps
them resident in HBM with the per-frame metadata, scoring query frames with the RAG engine's cosine
(rag/search/engine.py:622-660, on the extracted original embedding :604-620) or spatial-locality score
(:662-714) and ranking by (score desc, frame order asc).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .. import kernels as K
from .._dev import to_dev, to_np, torch
from . import similarity as S


@dataclass
class DocumentChunk:
    """rag/models.py:11-35 (same fields and validation)."""
    content: str
    ipfs_hash: str
    source_path: str
    start_position: int
    end_position: int
    chunk_sequence: int
    creation_timestamp: str
    chunk_size: int

    def __post_init__(self):
        if self.chunk_size <= 0:
            raise ValueError("Chunk size must be positive")
        if self.start_position < 0 or self.end_position < 0:
            raise ValueError("Positions must be non-negative")
        if self.start_position >= self.end_position:
            raise ValueError("Start position must be less than end position")
        if self.chunk_sequence < 0:
            raise ValueError("Chunk sequence must be non-negative")


@dataclass
class VideoFrameMetadata:
    """rag/models.py:62-83 (same fields and validation)."""
    frame_index: int
    chunk_id: str
    ipfs_hash: str
    source_document: str
    compression_quality: float
    hierarchical_indices: List[np.ndarray]
    embedding_model: str
    frame_timestamp: float
    chunk_metadata: DocumentChunk

    def __post_init__(self):
        if self.frame_index < 0:
            raise ValueError("Frame index must be non-negative")
        if self.compression_quality < 0 or self.compression_quality > 1:
            raise ValueError("Compression quality must be between 0 and 1")
        if self.frame_timestamp < 0:
            raise ValueError("Frame timestamp must be non-negative")


@dataclass
class DualStorageState:
    current_video_index: int = 0
    current_frame_count: int = 0
    frame_metadata: List[VideoFrameMetadata] = field(default_factory=list)


def load_dual_storage_metadata(storage_root: str = "rag_storage") -> DualStorageState:
    """rag/video_storage/dual_storage.py:51-84 `_load_existing_metadata` (the metadata directory is
    `<storage_root>/metadata`, :33-35)."""
    st = DualStorageState()
    metadata_file = os.path.join(storage_root, "metadata", "dual_video_metadata.json")
    if os.path.exists(metadata_file):
        try:
            with open(metadata_file, "r") as f:
                data = json.load(f)
                st.current_video_index = data.get("current_video_index", 0)
                st.current_frame_count = data.get("current_frame_count", 0)
                for frame_data in data.get("frame_metadata", []):
                    c = frame_data["chunk_metadata"]
                    chunk = DocumentChunk(content=c["content"], ipfs_hash=c["ipfs_hash"], source_path=c["source_path"],
                                          start_position=c["start_position"], end_position=c["end_position"],
                                          chunk_sequence=c["chunk_sequence"],
                                          creation_timestamp=c["creation_timestamp"], chunk_size=c["chunk_size"])
                    st.frame_metadata.append(VideoFrameMetadata(
                        frame_index=frame_data["frame_index"], chunk_id=frame_data["chunk_id"],
                        ipfs_hash=frame_data["ipfs_hash"], source_document=frame_data["source_document"],
                        compression_quality=frame_data["compression_quality"], hierarchical_indices=[],
                        embedding_model=frame_data["embedding_model"], frame_timestamp=frame_data["frame_timestamp"],
                        chunk_metadata=chunk))
        except Exception as e:
            print(f"Warning: Could not load existing metadata: {e}")
    return st


class DualStorageCorpus:
    """The dual storage's embedding frames [N, H, W] (decoded, in frame order) resident in HBM, with the
    frame metadata of `load_dual_storage_metadata`; query frames are scored on the GPU."""

    def __init__(self, frames, metadata: Sequence[VideoFrameMetadata]):
        x = to_dev(frames)
        if x.dim() != 3:
            raise ValueError("embedding frames must be [N, H, W]")
        if len(metadata) != int(x.shape[0]):
            raise ValueError(f"{int(x.shape[0])} frames for {len(metadata)} metadata entries")
        t = torch()
        self.frames = x if x.dtype in (t.float32, t.float64) else x.to(t.float64)
        self.metadata = list(metadata)
        self._cos = None

    @classmethod
    def from_storage(cls, storage_root: str, frames) -> "DualStorageCorpus":
        return cls(frames, load_dual_storage_metadata(storage_root).frame_metadata)

    def __len__(self) -> int:
        return len(self.metadata)

    def _originals(self, imgs):
        """Each image's rows above its detected index rows (engine.py:604-620), zero below, flattened;
        images whose heights differ score through the common prefix exactly as the reference's
        flatten-and-truncate cosine does only when the heights agree (checked by the caller)."""
        t = torch()
        h = torch().as_tensor(S.detect_original_embedding_heights(imgs), device=imgs.device)
        rows = t.arange(imgs.shape[1], device=imgs.device).view(1, -1, 1)
        return t.where(rows < h.view(-1, 1, 1), imgs, t.zeros((), dtype=imgs.dtype, device=imgs.device)), h

    def scores(self, query_frames, method: str = "spatial"):
        """Scores [Q, N] (device f64) of query frames [Q, H, W] against every stored frame:
        "spatial" = _calculate_spatial_locality_similarity (engine.py:662-714); "embedding" =
        _calculate_embedding_cosine_similarity of the extracted original embeddings (engine.py:604-660;
        a pair whose original heights differ compares flattened prefixes of different shapes, which the
        reference truncates to the shorter: such pairs are scored on their common flattened prefix)."""
        t = torch()
        q = to_dev(query_frames)
        q = (q.unsqueeze(0) if q.dim() == 2 else q).to(self.frames.dtype)
        if method == "spatial":
            return S.spatial_locality_scores(q, self.frames)
        if method != "embedding":
            raise ValueError(f"unknown method {method!r}")
        qo, qh = self._originals(q)
        co, ch = self._originals(self.frames)
        W = int(q.shape[2])
        out = t.empty((q.shape[0], self.frames.shape[0]), dtype=t.float64, device=q.device)
        for hq in t.unique(qh).tolist():
            qi = (qh == hq).nonzero().view(-1)
            for hc in t.unique(ch).tolist():
                ci = (ch == hc).nonzero().view(-1)
                m = min(hq, hc) * W   # the common flattened prefix
                s = K.cosine_scores_dt(qo[qi].reshape(len(qi), -1)[:, :m].contiguous(),
                                       co[ci].reshape(len(ci), -1)[:, :m].contiguous())
                out[qi.view(-1, 1), ci.view(1, -1)] = s
        return out

    def search(self, query_frames, k: int = 10, method: str = "spatial") -> List[List[Tuple[VideoFrameMetadata, float]]]:
        """Top-k stored frames per query by (score desc, frame order asc)."""
        sc = self.scores(query_frames, method)
        s, ids, _, _ = K.select_topk(sc, max(1, min(int(k), len(self))), 0.0, 0)
        s, ids = to_np(s), to_np(ids)
        return [[(self.metadata[int(i)], float(v)) for v, i in zip(s[r], ids[r]) if i >= 0] for r in range(len(s))]
