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


def test_frame_store_reference_written_metadata(hq_lib, tmp_path, golden):
    """The per-video JSON files written by the reference's own _save_video_metadata / _save_global_index
    (core/video_storage.py:579-631, tests/golden/make_golden.py `stores`), laid out in a directory: the
    loader reads the same frames, index vectors (bit-exact) and model -> (video, frame) map as the
    reference's _load_existing_index did, and the level-0 frame search ranks by the reference's own
    similarities in the directory's glob (visiting) order, ties included (duplicate rows across videos)."""
    from hq_mi355x.core.frame_store import FrameStoreCorpus
    g = golden("stores")
    for name, text in zip(g["video_json_names"], g["video_json_texts"]):
        (tmp_path / str(name)).write_text(str(text).replace("@STORE@", str(tmp_path)))
    store = FrameStoreCorpus.from_storage_dir(tmp_path)
    got = {fm.model_id: (vp, fm) for vp, fm in store.frames}
    ids = list(g["video_loaded_ids"])
    assert sorted(got, key=lambda s: int(s[1:])) == ids
    for k, m in enumerate(ids):
        vp, fm = got[m]
        assert fm.hierarchical_indices.tobytes() == g["video_loaded_idx"][k].tobytes()
        assert int(vp.rsplit("video_", 1)[1][0]) == g["video_loaded_map"][k][0] and fm.frame_index == g["video_loaded_map"][k][1]
    visit = [fm.model_id for _, fm in store.frames]          # glob order of this directory
    col = {m: i for i, m in enumerate(ids)}
    Q = g["video_queries"]
    res = store.hierarchical_search(Q, 10, 0.1)
    for a in range(len(Q)):
        sims = [g["video_sims"][a][col[m]] for m in visit]
        hits = sorted([(s, m) for s, m in zip(sims, visit) if s > 0.1], key=lambda h: h[0], reverse=True)[:10]
        assert [fm.model_id for fm, _ in res[a]] == [m for _, m in hits], a
        np.testing.assert_array_equal([s for _, s in res[a]], [s for s, _ in hits])


def test_rag_dual_storage_loader(hq_lib, tmp_path, golden):
    """RAG dual storage: dual_video_metadata.json written by the reference's own
    _save_metadata (rag/video_storage/dual_storage.py:86-121) is read back exactly as its
    _load_existing_metadata does (counters, frame and chunk fields, empty index lists); a broken file
    keeps the reference's warning-and-continue behaviour; the embedding frames, resident with that
    metadata, rank query frames by the RAG scorer (spatial locality and original-embedding cosine)
    like the oracle."""
    from hq_mi355x.rag.dual_storage import DualStorageCorpus, load_dual_storage_metadata
    g = golden("stores")
    (tmp_path / "metadata").mkdir()
    (tmp_path / "metadata" / "dual_video_metadata.json").write_text(str(g["dual_json_text"]))
    st = load_dual_storage_metadata(str(tmp_path))
    assert [st.current_video_index, st.current_frame_count] == list(g["dual_state"])
    got = [[str(f.frame_index), f.chunk_id, f.ipfs_hash, f.source_document, repr(f.compression_quality),
            f.embedding_model, repr(f.frame_timestamp), f.chunk_metadata.content, str(f.chunk_metadata.chunk_size)]
           for f in st.frame_metadata]
    assert got == [list(r) for r in g["dual_loaded"]]
    assert all(f.hierarchical_indices == [] for f in st.frame_metadata)
    assert load_dual_storage_metadata(str(tmp_path / "nowhere")).frame_metadata == []
    # frames: 12 enhanced 32 x 32 images (RAG index rows appended by the drop-in generator)
    from hq_mi355x.rag import HierarchicalIndexGenerator
    rng = np.random.default_rng(12)
    imgs = rng.standard_normal((12, 32, 32))
    imgs[5] = imgs[2] + 0.01 * rng.standard_normal((32, 32))
    gen = HierarchicalIndexGenerator()
    enh = np.stack([np.asarray(gen.generate_multi_level_indices(im)) for im in imgs])
    corpus = DualStorageCorpus.from_storage(str(tmp_path), enh)
    q = enh[[2, 7]]
    for method in ("spatial", "embedding"):
        res = corpus.search(q, 4, method)
        for a in range(2):
            if method == "spatial":
                want = np.array([O.rag_spatial_locality_enhanced(q[a], e) for e in enh])
            else:
                h = [O.rag_detect_height(e) for e in enh]
                hq_ = O.rag_detect_height(q[a])
                want = np.array([O.rag_cosine(q[a][:hq_].ravel(), e[:hc].ravel()[None])[0] for e, hc in zip(enh, h)])
            order = np.argsort(-want, kind="stable")[:4]
            assert [f.chunk_id for f, _ in res[a]] == [f"c{i}" for i in order], (method, a)
            np.testing.assert_allclose([s for _, s in res[a]], want[order], atol=1e-12)
    (tmp_path / "metadata" / "dual_video_metadata.json").write_text('{"current_video_index": 3, "frame_metadata": [{"x": 1}]}')
    st = load_dual_storage_metadata(str(tmp_path))   # prints the reference's warning, keeps the counters
    assert st.current_video_index == 3 and st.frame_metadata == []
