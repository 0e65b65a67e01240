"""End-to-end API parity with the reference: tests/golden/api.npz holds what the reference's own
HilbertQuantizer (api.py:120-297; core/pipeline.py:71-233; core/compressor.py:43-148, 256-303) produced
for seeded vectors (tests/golden/make_golden.py api_fixtures): the JPEG payload bytes, the hierarchical
indices, the compressor's de-normalisation state, every reconstruct() array and the search() rankings.
The per-model drop-in (HilbertQuantizer) and the batched ingest (BatchQuantizer) reproduce them: payloads
byte-identical (the same PIL encoder on the same frames), arrays bit-identical, rankings identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DIMS = [1024, 3000, 4096]


def _ids(results):
    return [int(x.model.metadata.model_name.rsplit("_m", 1)[1]) for x in results]


def _check_models(g, tag, models):
    for i, m in enumerate(models):
        assert m.compressed_data == g[f"{tag}_payload_{i}"].tobytes(), (tag, i)
        want = g[f"{tag}_hidx_{i}"]
        assert m.hierarchical_indices.dtype == want.dtype
        np.testing.assert_array_equal(m.hierarchical_indices, want)
        assert tuple(m.original_dimensions) == tuple(g[f"{tag}_dims"][i])
        assert m.parameter_count == int(g[f"{tag}_count"][i])
        assert m.compression_quality == float(g[f"{tag}_quality"][i])


def _check_search(g, tag, got):
    for a, r in enumerate(got):
        want = [i for i in g[f"{tag}_search_ids"][a] if i >= 0]
        assert _ids(r) == want, (tag, a)
        np.testing.assert_array_equal([x.similarity_score for x in r], g[f"{tag}_search_sc"][a][: len(r)])
        np.testing.assert_array_equal([x.reconstruction_error for x in r], g[f"{tag}_search_err"][a][: len(r)])


@pytest.mark.parametrize("d", DIMS)
def test_hilbert_quantizer_end_to_end_golden(hq_lib, golden, d):
    from hq_mi355x.api import HilbertQuantizer
    g = golden("api")
    tag = f"d{d}"
    P = g[f"{tag}_params"]
    hqz = HilbertQuantizer(use_precomputed_indexing=True)
    models = [hqz.quantize(P[i], model_id=f"{tag}_m{i}") for i in range(8)]
    _check_models(g, tag, models)
    comp = hqz.quantization_pipeline.compressor
    np.testing.assert_array_equal([comp._norm_min, comp._norm_max], g[f"{tag}_minmax_last"])
    recon = np.stack([hqz.reconstruct(m) for m in models])
    assert recon.dtype == g[f"{tag}_recon"].dtype
    np.testing.assert_array_equal(recon, g[f"{tag}_recon"])
    Qs = g[f"{tag}_queries"]
    _check_search(g, tag, [hqz.search(Qs[a], candidate_models=models, max_results=8) for a in range(len(Qs))])


@pytest.mark.parametrize("d", DIMS)
def test_batch_quantizer_end_to_end_golden(hq_lib, golden, d):
    from hq_mi355x.api import BatchQuantizer
    g = golden("api")
    tag = f"d{d}"
    P = g[f"{tag}_params"]
    bq = BatchQuantizer()
    models = bq.quantize_batch(list(P), model_ids=[f"{tag}_m{i}" for i in range(8)])
    _check_models(g, tag, models)
    recon = np.stack(bq.reconstruct_batch(models))
    np.testing.assert_array_equal(recon, g[f"{tag}_recon"])
    _check_search(g, tag, bq.search_batch(list(g[f"{tag}_queries"]), models, max_results=8))


def test_efficiency_refusal_golden(hq_lib, golden):
    """1536 values on a 64 x 64 grid (efficiency 0.375 < 0.5): the reference's exception and text."""
    from hq_mi355x.api import HilbertQuantizer
    g = golden("api")
    with pytest.raises(Exception) as ei:
        HilbertQuantizer(use_precomputed_indexing=True).quantize(
            np.random.default_rng(0).standard_normal(1536).astype(np.float32), model_id="eff")
    assert f"{type(ei.value).__name__}: {ei.value}" == str(g["d1536_error"])
