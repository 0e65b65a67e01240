"""Frame-store loader: the reference's video-storage metadata files straight into
a device-resident search corpus.

The reference's VideoModelStorage writes one JSON file per video next to it
(core/video_storage.py:579-631, `_save_video_metadata`: `frame_metadata[*].hierarchical_indices` as
`ndarray.tolist()` of float64, which JSON round-trips exactly) plus a global `video_index.json`, and
reads them back in `_load_existing_index` (:633-691) in `Path.glob("*.json")` order.  The level-0
frame search (`_hierarchical_search`, core/video_search.py:215-264) then visits
`_video_index.values()` → `frame_metadata` in that insertion order, so candidate order — which
decides the stable-sort tie order — is (file in glob order, frame in file order).  `FrameStoreCorpus`
keeps exactly that order, uploads all index vectors once, and answers query batches with one launch
(`IndexCorpus.frame_search`, strict `> threshold`, or the progressive search).
"""
from __future__ import annotations

import json
import logging
from dataclasses import dataclass
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .._dev import to_np
from ..models import ModelMetadata
from .search_engine import IndexCorpus

logger = logging.getLogger(__name__)


@dataclass
class VideoFrameMetadata:
    """core/video_storage.py:29-39 (fields read back from the JSON index)."""
    frame_index: int
    model_id: str
    original_parameter_count: int
    compression_quality: float
    hierarchical_indices: np.ndarray
    model_metadata: ModelMetadata
    frame_timestamp: float
    similarity_features: Optional[np.ndarray] = None


def load_video_metadata(json_path) -> Tuple[str, List[VideoFrameMetadata]]:
    """One per-video metadata file (core/video_storage.py:633-664) -> (video_path, frames in order)."""
    with open(json_path, "r") as f:
        d = json.load(f)
    frames = []
    for fm in d["frame_metadata"]:
        frames.append(VideoFrameMetadata(
            frame_index=fm["frame_index"], model_id=fm["model_id"],
            original_parameter_count=fm["original_parameter_count"], compression_quality=fm["compression_quality"],
            hierarchical_indices=np.array(fm["hierarchical_indices"]), model_metadata=ModelMetadata(**fm["model_metadata"]),
            frame_timestamp=fm["frame_timestamp"],
            similarity_features=np.array(fm["similarity_features"]) if fm["similarity_features"] else None))
    return d["video_path"], frames


class FrameStoreCorpus:
    """All frames of a storage directory as one IndexCorpus (rows in the reference's visiting order)."""

    def __init__(self, frames: Sequence[Tuple[str, VideoFrameMetadata]], id_base: int = 0):
        if not frames:
            raise ValueError("No frames found in video storage")
        lens = {len(fm.hierarchical_indices) for _, fm in frames}
        if len(lens) != 1:
            raise ValueError(f"frames carry index vectors of different lengths {sorted(lens)}")
        self.frames = list(frames)
        self.corpus = IndexCorpus(np.stack([np.asarray(fm.hierarchical_indices, dtype=np.float64)
                                            for _, fm in self.frames]), id_base)

    @classmethod
    def from_storage_dir(cls, storage_dir, id_base: int = 0) -> "FrameStoreCorpus":
        videos: Dict[str, List[VideoFrameMetadata]] = {}  # the reference's _video_index (dict semantics)
        for json_file in Path(storage_dir).glob("*.json"):
            if json_file.name == "video_index.json":
                continue
            try:
                video_path, fl = load_video_metadata(json_file)
            except Exception as e:  # the reference logs and skips unreadable files (:690-691)
                logger.error(f"Failed to load metadata from {json_file}: {e}")
                continue
            videos[video_path] = fl
        frames = [(vp, fm) for vp, fl in videos.items() for fm in fl]
        return cls(frames, id_base)

    def __len__(self) -> int:
        return len(self.frames)

    def hierarchical_search(self, query_indices, max_results: int, similarity_threshold: float = 0.1):
        """`_hierarchical_search` for a batch of query index vectors [Q, L] -> per query a list of
        (VideoFrameMetadata, similarity) in the reference's order (sim > threshold, stable desc)."""
        q = np.asarray(query_indices, dtype=np.float64)
        if q.ndim == 1:
            q = q[None]
        ids, sc = self.corpus.frame_search(q, max_results, similarity_threshold)
        ids, sc = to_np(ids), to_np(sc)
        base = self.corpus.id_base
        return [[(self.frames[int(i) - base][1], float(s)) for i, s in zip(ids[r], sc[r]) if i >= 0]
                for r in range(len(q))]
