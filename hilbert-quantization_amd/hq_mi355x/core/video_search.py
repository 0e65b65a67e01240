"""Level-0 scan over stored frames: the `hierarchical` mode of the
reference's VideoEnhancedSearchEngine (core/video_search.py:215-264, :1316-1328), which compares the
query's index with every stored frame's `hierarchical_indices` at level 0, keeps sim > threshold
(strict), and stable-sorts descending.  Frames are held as one device-resident IndexCorpus."""
from __future__ import annotations

from typing import List, Sequence, Tuple


from .._dev import to_np
from .search_engine import IndexCorpus, _idx


class HierarchicalFrameSearch:
    def __init__(self, frame_indices, similarity_threshold: float = 0.1):
        self.corpus = IndexCorpus(frame_indices)
        self.similarity_threshold = similarity_threshold

    def search(self, query_indices, max_results: int) -> List[Tuple[int, float]]:
        # the query keeps its dtype: a float32 index is compared with float32 statistics, as in the reference
        ids, sc = self.corpus.frame_search(_idx(query_indices)[None], max_results, self.similarity_threshold)
        ids, sc = to_np(ids)[0], to_np(sc)[0]
        return [(int(i), float(s)) for i, s in zip(ids, sc) if i >= 0]

    def search_batch(self, queries, max_results: int):
        return self.corpus.frame_search(queries, max_results, self.similarity_threshold)
