"""Batched QuantizedModel ingest: BatchQuantizer / HilbertQuantizer.quantize_many
produce the same models, registry, pre-computed indices, compressor state and errors as calling
HilbertQuantizer.quantize model by model (api.py:120-186, :567-650)."""
import contextlib
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sets(rng):
    sets = [rng.standard_normal(1024).astype(np.float32) for _ in range(5)]
    sets.insert(2, rng.standard_normal(4096).astype(np.float32) * 3)
    sets.append(np.full(1024, 0.5, dtype=np.float32))            # constant: compressor state untouched
    sets.append(rng.standard_normal(256).astype(np.float32))
    return sets


def test_batch_quantize_matches_sequential(hq_lib):
    pytest.importorskip("PIL")
    from hq_mi355x.api import BatchQuantizer, HilbertQuantizer
    rng = np.random.default_rng(3)
    sets = _sets(rng)
    ids = [f"m{i}" for i in range(len(sets))]
    seq = HilbertQuantizer()
    with contextlib.redirect_stdout(io.StringIO()):
        want = [seq.quantize(p, model_id=m) for p, m in zip(sets, ids)]
    bq = BatchQuantizer()
    got = bq.quantize_batch(sets, model_ids=ids)
    assert [m.metadata.model_name for m in bq.quantizer._model_registry] == ids
    for a, b in zip(got, want):
        assert a.compressed_data == b.compressed_data
        assert a.hierarchical_indices.tobytes() == b.hierarchical_indices.tobytes()
        assert a.original_dimensions == b.original_dimensions and a.parameter_count == b.parameter_count
        assert (a.metadata.original_size_bytes, a.metadata.compressed_size_bytes) == \
            (b.metadata.original_size_bytes, b.metadata.compressed_size_bytes)
        pa = bq.quantizer.precomputed_indexer.get_index(a.metadata.model_name)
        pb = seq.precomputed_indexer.get_index(b.metadata.model_name)
        assert all(x.averages.tobytes() == y.averages.tobytes() for x, y in zip(pa.levels, pb.levels))
        assert pa.total_storage_bytes == pb.total_storage_bytes
    c1, c2 = bq.quantizer.quantization_pipeline.compressor, seq.quantization_pipeline.compressor
    assert (c1._norm_min, c1._norm_max) == (c2._norm_min, c2._norm_max)
    # reconstruct through the drop-in round trip works on batch-made models
    rec = bq.quantizer.reconstruct(got[0])
    assert rec.shape == (1024,)


def test_batch_quantize_first_failure_order(hq_lib):
    pytest.importorskip("PIL")
    from hq_mi355x.api import BatchQuantizer
    from hq_mi355x.exceptions import QuantizationError, ValidationError
    rng = np.random.default_rng(4)
    sets = [rng.standard_normal(1024).astype(np.float32) for _ in range(2)]
    bad = rng.standard_normal(1536).astype(np.float32)
    bq = BatchQuantizer()
    with pytest.raises(QuantizationError, match="Failed to quantize model 'model_2': Efficiency ratio 0.375"):
        bq.quantize_batch(sets + [bad] + sets)
    assert len(bq.quantizer._model_registry) == 2
    nan = sets[0].copy()
    nan[3] = np.nan
    bq2 = BatchQuantizer()
    with pytest.raises(ValidationError, match="non-finite"):
        bq2.quantize_batch([sets[0], nan, sets[1]])
    assert [m.metadata.model_name for m in bq2.quantizer._model_registry] == ["model_0"]
    with pytest.raises(ValueError, match="Number of model IDs must match"):
        bq.quantize_batch(sets, model_ids=["a"])


def test_search_batch_matches_sequential(hq_lib):
    pytest.importorskip("PIL")
    from hq_mi355x.api import BatchQuantizer, HilbertQuantizer
    rng = np.random.default_rng(5)
    base = [rng.standard_normal(1024).astype(np.float32) for _ in range(40)]
    bq = BatchQuantizer()
    cands = bq.quantize_batch(base)
    queries = [base[i] + rng.normal(0, 0.05, 1024).astype(np.float32) for i in (0, 7, 21)]
    queries.append(np.zeros(0, dtype=np.float32))   # invalid query -> []
    got = bq.search_batch(queries, cands, max_results=5)
    seq = HilbertQuantizer()
    for q, res in zip(queries, got):
        if q.size == 0:
            assert res == []
            continue
        with contextlib.redirect_stdout(io.StringIO()):
            want = seq.search(q, cands, max_results=5)
        assert [r.model.metadata.model_name for r in res] == [r.model.metadata.model_name for r in want]
        assert [r.similarity_score for r in res] == [r.similarity_score for r in want]
        assert [r.matching_indices for r in res] == [r.matching_indices for r in want]
    # the queries were registered, as search() does
    assert len(bq.quantizer._model_registry) == 40 + 3


def test_search_batch_failing_query_only_blanks_itself(hq_lib):
    """a query failing the efficiency check (api.py:621-650 catches per query) yields []
    while the queries before AND after it are quantized, registered and answered."""
    pytest.importorskip("PIL")
    from hq_mi355x.api import BatchQuantizer, HilbertQuantizer
    rng = np.random.default_rng(8)
    base = [rng.standard_normal(1024).astype(np.float32) for _ in range(30)]
    bq = BatchQuantizer()
    cands = bq.quantize_batch(base)
    bad = rng.standard_normal(1500).astype(np.float32)  # 1500 / 4096 < 0.5: QuantizationError
    queries = [base[2] + np.float32(0.01), bad, base[9] + np.float32(0.02), bad, base[17] + np.float32(0.03)]
    got = bq.search_batch(queries, cands, max_results=5)
    assert got[1] == [] and got[3] == []
    seq = HilbertQuantizer()
    for i in (0, 2, 4):
        with contextlib.redirect_stdout(io.StringIO()):
            want = seq.search(queries[i], cands, max_results=5)
        assert got[i], i
        assert [r.model.metadata.model_name for r in got[i]] == [r.model.metadata.model_name for r in want]
        assert [r.similarity_score for r in got[i]] == [r.similarity_score for r in want]
    assert len(bq.quantizer._model_registry) == 30 + 3


def test_batched_reconstruct_matches_per_model(hq_lib):
    """HilbertQuantizer.reconstruct_many (host JPEG decode on threads, one de-normalise
    and one inverse-Hilbert gather per frame shape) returns exactly reconstruct()'s arrays, model by model,
    including the reference's quirk of de-normalising with the compressor's LAST (min, max)
    (core/compressor.py:282-303, core/pipeline.py:183-235); mixed vector lengths; bad payloads raise the
    per-model errors."""
    pytest.importorskip("PIL")
    from hq_mi355x.api import BatchQuantizer, HilbertQuantizer
    from hq_mi355x.exceptions import ReconstructionError
    rng = np.random.default_rng(9)
    sets = _sets(rng)
    hq = HilbertQuantizer()
    models = hq.quantize_many(sets, model_ids=[f"r{i}" for i in range(len(sets))])
    want = [hq.reconstruct(m) for m in models]
    got = hq.reconstruct_many(models)
    assert len(got) == len(want)
    for a, b, p in zip(got, want, sets):
        assert a.dtype == b.dtype and a.shape == b.shape == p.shape
        assert a.tobytes() == b.tobytes()
    got2 = BatchQuantizer().reconstruct_batch(models)   # fresh compressor: u8 / 255 (no state)
    fresh = HilbertQuantizer()
    for a, m in zip(got2, models):
        assert a.tobytes() == fresh.reconstruct(m).tobytes()
    import dataclasses
    bad = dataclasses.replace(models[0], compressed_data=b"\x00\x01not a jpeg")
    with pytest.raises(ReconstructionError, match="Failed to decompress image"):
        hq.reconstruct_many([models[1], bad])
    with pytest.raises(ReconstructionError, match="Failed to decompress image"):
        hq.reconstruct(bad)
