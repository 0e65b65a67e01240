"""Frame-store loader: the reference's per-video JSON metadata
(core/video_storage.py:579-691) into one device corpus; level-0 frame search in the reference's
candidate order (core/video_search.py:215-264) against the oracle."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu


def _write_video(path: Path, video_path: str, idx: np.ndarray, first_id: int):
    md = {"model_name": "x", "original_size_bytes": 4096, "compressed_size_bytes": 512, "compression_ratio": 8.0,
          "quantization_timestamp": "2025-01-01 00:00:00", "model_architecture": None, "additional_info": {}}
    d = {"video_path": video_path, "total_frames": len(idx), "frame_rate": 30.0, "video_codec": "mp4v",
         "frame_dimensions": [65, 64], "creation_timestamp": "2025-01-01 00:00:00",
         "last_modified_timestamp": "2025-01-01 00:00:00", "video_file_size_bytes": 0,
         "total_models_stored": len(idx), "average_compression_ratio": 8.0, "video_index_version": "1.0",
         "frame_metadata": [{"frame_index": i, "model_id": f"m{first_id + i}", "original_parameter_count": 1536,
                             "compression_quality": 0.8, "hierarchical_indices": idx[i].tolist(),
                             "frame_timestamp": 0.0, "similarity_features": None, "model_metadata": dict(md)}
                            for i in range(len(idx))]}
    path.write_text(json.dumps(d, indent=2))


def test_frame_store_search_vs_oracle(hq_lib, tmp_path):
    from hq_mi355x.core.frame_store import FrameStoreCorpus
    rng = np.random.default_rng(6)
    C = rng.standard_normal((3 * 40, 64)).cumsum(1) * 0.1
    C[45] = C[3]                       # duplicates across videos: ties keep the visiting order
    C[90] = C[3]
    for v in range(3):
        _write_video(tmp_path / f"video_{v}.json", f"{tmp_path}/video_{v}.mp4", C[40 * v:40 * (v + 1)], 40 * v)
    (tmp_path / "video_index.json").write_text("{}")
    (tmp_path / "broken.json").write_text("{not json")   # skipped with an error log, like the reference
    store = FrameStoreCorpus.from_storage_dir(tmp_path)
    assert len(store) == 120
    order = [fm.model_id for _, fm in store.frames]
    # the reference's visiting order: Path.glob order of the files, frames in file order
    want_order = []
    for f in Path(tmp_path).glob("*.json"):
        if f.name in ("video_index.json", "broken.json"):
            continue
        want_order += [fm["model_id"] for fm in json.loads(f.read_text())["frame_metadata"]]
    assert order == want_order
    Cv = np.stack([fm.hierarchical_indices for _, fm in store.frames])
    assert Cv.tobytes() == np.stack([C[int(m[1:])] for m in order]).tobytes()   # exact JSON round trip
    Q = np.stack([C[3] + 0.0, C[17] + rng.normal(0, 0.01, 64), C[100] + rng.normal(0, 0.05, 64)])
    got = store.hierarchical_search(Q, 10, 0.1)
    for q, res in zip(Q, got):
        pos, sc = O.hierarchical_frame_search(q, Cv, 10, 0.1)
        assert [fm.model_id for fm, _ in res] == [order[p] for p in pos]
        assert [s for _, s in res] == list(sc)
