"""GPU parity: Hilbert maps (M1-M6), indices (I1, I2, I4), uint8 quantize (Q1, Q2) and the fused
north-star kernel against the reference golden vectors and the CPU oracle.  Bit-exact throughout."""
import numpy as np
import pytest

from oracle import hq_oracle as O

pytestmark = pytest.mark.gpu


def _t(x):
    from hq_mi355x._dev import to_dev
    return to_dev(x)


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def test_native_library_loaded(hq_lib):
    import hq_mi355x._lib as L
    assert hq_lib.hq_version() == 1
    assert L.LIB_PATH.endswith("libhq_mi355x.so")


# ------------------------------------------------------------------------------------------ maps


def test_tables_golden(hq_lib, golden):
    from hq_mi355x import kernels as K
    g = golden("mapper")
    for n in [1, 2, 4, 8, 16, 32, 64, 128]:
        xs, ys, tab = K.hilbert_table(n)
        np.testing.assert_array_equal(np.stack([_np(xs), _np(ys)], 1), g[f"coords_n{n}"])
        if f"xy2d_n{n}" in g:
            np.testing.assert_array_equal(_np(tab), g[f"xy2d_n{n}"])


def test_dropin_mapper_golden(hq_lib, golden):
    from hq_mi355x.core import HilbertCurveMapper
    from hq_mi355x.rag import HilbertCurveMapperImpl
    from hq_mi355x.exceptions import HilbertQuantizationError
    m, rm = HilbertCurveMapper(), HilbertCurveMapperImpl()
    g = golden("mapper")
    k = 0
    while f"map_in_{k}" in g:
        p, img = g[f"map_in_{k}"], g[f"map_out_{k}"]
        n = img.shape[0]
        out = m.map_to_2d(p, (n, n))
        assert out.dtype == img.dtype and out.tobytes() == img.tobytes()
        assert rm.map_to_2d(p, (n, n)).tobytes() == g[f"rag_map_out_{k}"].tobytes()
        un = m.map_from_2d(img)
        assert un.dtype == img.dtype and un.tobytes() == g[f"unmap_out_{k}"].tobytes()
        k += 1
    # reference KATs (tests/test_hilbert_mapper.py:23,43-46,102-120,173-182)
    assert m.generate_hilbert_coordinates(2) == [(0, 0), (0, 1), (1, 1), (1, 0)]
    assert m.generate_hilbert_coordinates(4)[:4] == [(0, 0), (1, 0), (1, 1), (0, 1)]
    assert list(m.map_from_2d(np.array([[1, 4], [2, 3]]))) == [1, 2, 3, 4]
    assert list(rm.map_from_2d(np.array([[1, 2], [3, 4]]))) == [1, 3, 4, 2]
    for i in range(16):
        x, y = m._hilbert_index_to_xy(i, 4)
        assert m._xy_to_hilbert_index(x, y, 4) == i
    with pytest.raises(HilbertQuantizationError, match="square dimensions, got 4x8"):
        m.map_to_2d(np.zeros(4, np.float32), (4, 8))
    with pytest.raises(HilbertQuantizationError, match="power of 2, got 6"):
        m.map_to_2d(np.zeros(4, np.float32), (6, 6))
    with pytest.raises(HilbertQuantizationError, match=r"Too many parameters \(17\) for dimensions 4x4 \(16 cells\)"):
        m.map_to_2d(np.zeros(17, np.float32), (4, 4))
    with pytest.raises(ValueError, match="Too many embedding values"):
        rm.map_to_2d(np.zeros(17, np.float32), (4, 4))
    with pytest.raises(ValueError, match="Input must be 2D array, got 1D"):
        rm.map_from_2d(np.zeros(4))
    # empty input: all-zero image
    assert not m.map_to_2d(np.zeros(0, np.float32), (4, 4)).any()


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.float16, np.int32, np.int64, np.uint8])
def test_batched_maps_vs_oracle(hq_lib, dtype):
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(11)
    for n, d, N in [(2, 3, 5), (8, 64, 7), (32, 1000, 33), (64, 1536, 65), (128, 16384, 3), (256, 40000, 2)]:
        P = (rng.standard_normal((N, d)) * 100).astype(dtype)
        img = K.map_to_2d(_t(P), n)
        ref = O.map_to_2d(P, n)
        assert _np(img).tobytes() == ref.tobytes()
        back = K.map_from_2d(img, d)
        assert _np(back).tobytes() == P.tobytes()          # round trip (size-independent property)
        assert _np(K.map_from_2d(img)).tobytes() == O.map_from_2d(ref).tobytes()


def test_strided_rows(hq_lib):
    from hq_mi355x import kernels as K
    import torch
    x = torch.randn(9, 2000, device="cuda")
    sub = x[:, 100:1636]
    img = K.map_to_2d(sub, 64)
    ref = O.map_to_2d(sub.cpu().numpy(), 64)
    assert _np(img).tobytes() == ref.tobytes()


# --------------------------------------------------------------------------------------- indices


def test_streaming_index_golden(hq_lib, golden):
    from hq_mi355x.core import StreamingHilbertIndexGenerator
    gen = StreamingHilbertIndexGenerator()
    g = golden("index")
    k = 0
    while f"stream_img_{k}" in g:
        got = gen.generate_optimized_indices(g[f"stream_img_{k}"], int(g[f"stream_L_{k}"]))
        assert got.dtype == np.float64 and got.tobytes() == g[f"stream_idx_{k}"].tobytes(), k
        k += 1
    with pytest.raises(ValueError, match="power-of-2 dimensions, got 6x6"):
        gen.generate_optimized_indices(np.zeros((6, 6)), 4)


def test_streaming_during_mapping_partial_groups(hq_lib):
    from hq_mi355x.core import StreamingHilbertIndexGenerator
    gen = StreamingHilbertIndexGenerator()
    rng = np.random.default_rng(4)
    for d, n, L in [(1000, 32, 32), (1537, 64, 64), (30, 8, 10), (5, 4, 3)]:
        p = rng.standard_normal(d).astype(np.float32)
        img, idx, _ = gen.generate_indices_during_mapping(p, (n, n), L)
        ref = O.streaming_index(p, L)   # the builder only sees the d real values (:287-313)
        assert idx.tobytes() == ref.tobytes(), (d, n, L)


def test_traditional_and_rag_golden(hq_lib, golden):
    from hq_mi355x.core import HierarchicalIndexGeneratorImpl
    from hq_mi355x.rag import HierarchicalIndexGenerator
    g = golden("index")
    tg = HierarchicalIndexGeneratorImpl()
    k = 0
    while f"trad_img_{k}" in g:
        got = tg.generate_optimized_indices(g[f"trad_img_{k}"], int(g[f"trad_L_{k}"]))
        assert got.dtype == np.float32 and got.tobytes() == g[f"trad_idx_{k}"].tobytes(), k
        k += 1
    rg = HierarchicalIndexGenerator()
    for k in range(5):
        img, ref = g[f"rag_img_{k}"], g[f"rag_rows_{k}"]
        got = rg.generate_multi_level_indices(img)
        assert got.dtype == ref.dtype and got.tobytes() == ref.tobytes(), k
    img = g["trad_img_2"]
    for grid in [1, 2, 4, 8, 64]:
        assert tg.calculate_spatial_averages(img, grid) == [float(v) for v in O.spatial_averages(img[None], grid)[0]]


def test_indices_vs_oracle_random(hq_lib):
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(21)
    for n, L in [(4, 4), (16, 16), (32, 32), (64, 64), (64, 17), (128, 128), (32, 100)]:
        imgs = (rng.standard_normal((6, n, n)) * 5 + 1).astype(np.float32)
        got = _np(K.index_streaming(_t(imgs), L))
        assert got.tobytes() == O.streaming_index(O.map_from_2d(imgs), L).tobytes()
        got = _np(K.index_traditional(_t(imgs), L))
        assert got.tobytes() == O.traditional_index(imgs, L).tobytes(), (n, L)
        got = _np(K.index_rag(_t(imgs)))
        assert got.tobytes() == O.rag_multi_level_indices(imgs).tobytes()


# -------------------------------------------------------------------------------------- quantize


def test_fused_kernel_golden(hq_lib, golden):
    from hq_mi355x.core.pipeline import quantize_batch
    g = golden("quant")
    for tag in ["d1536", "d1024", "d300", "d4096"]:
        P = g[f"{tag}_params"]
        fr, idx, mm = quantize_batch(P, min_efficiency_ratio=0.2)
        assert _np(fr).tobytes() == g[f"{tag}_frames"].tobytes(), tag
        assert _np(idx).tobytes() == g[f"{tag}_idx"].tobytes(), tag
        assert _np(mm)[:, 0].tobytes() == g[f"{tag}_min"].tobytes()
        assert _np(mm)[:, 1].tobytes() == g[f"{tag}_max"].tobytes()


def _oracle_fused(P, n, L):
    img = O.map_to_2d(O.pad_parameters(P, n), n)
    idx = O.streaming_index(O.map_from_2d(img), L)
    enh = O.embed_index_row(img, idx)
    u8, mn, mx = O.normalize_u8(enh)
    return u8, idx, mn, mx


@pytest.mark.parametrize("n,d,L", [(2, 3, 2), (4, 16, 4), (8, 33, 8), (16, 200, 16), (32, 1024, 32),
                                   (32, 999, 20), (64, 1536, 64), (64, 4096, 64), (64, 2049, 100),
                                   (128, 16384, 128), (128, 9000, 5)])
def test_fused_kernel_vs_oracle(hq_lib, n, d, L):
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(n * 1000 + d)
    P = (rng.standard_normal((37, d)) * rng.uniform(0.1, 10)).astype(np.float32)
    P[3] = 0.0                          # constant (all padding value) -> 128 frame
    P[4] = 2.5                          # constant non-zero
    P[5, :] = np.abs(P[5, :]) + 1.0     # strictly positive data, min from the zero padding
    fr, idx, mm = K.map_index_quantize(_t(P), n, L)
    u8, ridx, mn, mx = _oracle_fused(P, n, L)
    assert _np(fr).tobytes() == u8.tobytes()
    assert _np(idx).tobytes() == ridx.tobytes()
    got = _np(mm)
    assert np.array_equal(got[:, 0], mn) and np.array_equal(got[:, 1], mx)


@pytest.mark.parametrize("variant", [4, 0, 64, 192, 320, 448, 322, 576, 704, 832, 706, 1728, 3776])
@pytest.mark.parametrize("n,d,L", [(64, 1536, 64), (32, 999, 20), (16, 200, 16)])
def test_fused_launch_forms_vs_oracle(hq_lib, n, d, L, variant, hq_option):
    """Every launch form of the fast kernel (persistent triple/double buffered, non-persistent with 1-8
    waves per workgroup and a ragged last workgroup, reciprocal quantize) is bit-exact."""
    from hq_mi355x import kernels as K
    hq_option("fused_v", variant)
    rng = np.random.default_rng(variant + d)
    P = (rng.standard_normal((45, d)) * 3).astype(np.float32)
    P[7] = 0.0
    fr, idx, mm = K.map_index_quantize(_t(P), n, L)
    u8, ridx, mn, mx = _oracle_fused(P, n, L)
    assert _np(fr).tobytes() == u8.tobytes()
    assert _np(idx).tobytes() == ridx.tobytes()
    got = _np(mm)
    assert np.array_equal(got[:, 0], mn) and np.array_equal(got[:, 1], mx)


@pytest.mark.parametrize("n,d,L", [(32, 1000, 32), (64, 1536, 64), (64, 4096, 30), (16, 256, 16)])
def test_fused_generic_path_vs_oracle(hq_lib, n, d, L, hq_option):
    """The non-pipelined kernel (n outside {16,32,64}, L > 64, unaligned rows) stays bit-exact too."""
    from hq_mi355x import kernels as K
    hq_option("fused_generic", 1)
    rng = np.random.default_rng(d + L)
    P = rng.standard_normal((19, d)).astype(np.float32)
    fr, idx, mm = K.map_index_quantize(_t(P), n, L)
    u8, ridx, mn, mx = _oracle_fused(P, n, L)
    assert _np(fr).tobytes() == u8.tobytes()
    assert _np(idx).tobytes() == ridx.tobytes()


def test_fused_unaligned_rows(hq_lib):
    """Row stride not a multiple of 4 floats: the fast path declines, results still exact."""
    from hq_mi355x import kernels as K
    import torch
    x = torch.randn(23, 1537, device="cuda")
    sub = x[:, :1536]
    fr, idx, _ = K.map_index_quantize(sub, 64, 64)
    u8, ridx, _, _ = _oracle_fused(sub.cpu().numpy(), 64, 64)
    assert _np(fr).tobytes() == u8.tobytes() and _np(idx).tobytes() == ridx.tobytes()


def test_quantize_dequantize_vs_oracle(hq_lib, golden):
    from hq_mi355x.core import MPEGAICompressorImpl
    from hq_mi355x import kernels as K
    rng = np.random.default_rng(8)
    E = (rng.standard_normal((11, 65, 64)) * 3).astype(np.float32)
    E[2] = 7.0
    u8, mm = K.quantize_u8(_t(E))
    ru8, rmn, rmx = O.normalize_u8(E)
    assert _np(u8).tobytes() == ru8.tobytes()
    de = _np(K.dequantize_u8(u8, mm))
    for i in range(len(E)):
        assert de[i].tobytes() == O.denormalize_u8(ru8[i], rmn[i], rmx[i]).tobytes()
    # drop-in compressor keeps the reference's instance-state semantics (core/compressor.py:256-303)
    c = MPEGAICompressorImpl()
    g = golden("quant")
    assert c._normalize_for_compression(np.full((5, 4), 2.5, np.float32)).tobytes() == g["const_frame"].tobytes()
    assert not hasattr(c, "_norm_min")
    assert np.array_equal(c._denormalize_from_compression(np.full((2, 2), 128, np.uint8)),
                          np.full((2, 2), np.float32(128) / np.float32(255.0)))
    c._normalize_for_compression(E[0])
    assert c._denormalize_from_compression(ru8[0]).tobytes() == O.denormalize_u8(ru8[0], rmn[0], rmx[0]).tobytes()


def test_chunk_encoder_vs_oracle(hq_lib):
    from hq_mi355x import kernels as K
    import torch
    rng = np.random.default_rng(5)
    total = 1024 * 37 + 600
    x = (rng.standard_normal(total) * 0.02).astype(np.float16)
    fr, idx, mm = K.chunk_encode_f16(_t(x), 1024)
    fr, idx, mm = _np(fr), _np(idx), _np(mm)
    for c in range(38):
        chunk = x[c * 1024:(c + 1) * 1024].astype(np.float32)   # astype(float32) (:581)
        n = O.optimal_dimensions(len(chunk))[0]
        img = O.map_to_2d(chunk, n)
        ridx = O.traditional_index(img, n)
        u8, mn, mx = O.normalize_u8(O.embed_index_row(img, ridx))
        assert fr[c][: n + 1, :n].tobytes() == u8.tobytes(), c
        assert idx[c][:n].tobytes() == ridx.tobytes(), c
        assert mm[c, 0] == mn and mm[c, 1] == mx


@pytest.mark.parametrize("chunk,nfull,tail", [(1024, 41, 512), (4096, 9, 2500), (1024, 8, 0)])
@pytest.mark.parametrize("mode", ["fast", "exactdiv", "generic", "cpw1", "cpw4", "wpb2"])
def test_chunk_encoder_shapes_vs_oracle(hq_lib, chunk, nfull, tail, mode, hq_option):
    """Fast (one chunk per wave) and generic chunk kernels: odd chunk counts (a dead wave in the last
    workgroup), 64 x 64 chunks, the cfg5 512-value tail, constant chunks, caller-provided buffers."""
    from hq_mi355x import kernels as K
    import torch
    if mode == "generic":
        hq_option("chunk_generic", 1)
    if mode == "exactdiv":
        hq_option("chunk_exactdiv", 1)
    if mode in ("cpw1", "cpw4"):
        hq_option("chunk_cpw", int(mode[-1]))
    if mode == "wpb2":
        hq_option("chunk_wpb", 2)
    rng = np.random.default_rng(chunk + nfull)
    total = chunk * nfull + tail
    x = (rng.standard_normal(total) * 0.02).astype(np.float16)
    x[chunk:2 * chunk] = np.float16(0.5)          # constant chunk -> all 128
    x[2 * chunk + 7] = np.float16(-65504.0)       # extreme value
    n = O.optimal_dimensions(chunk)[0]
    nch = nfull + (1 if tail else 0)
    out = (torch.full((nch, n + 1, n), 7, dtype=torch.uint8, device="cuda"),
           torch.zeros((nch, n), dtype=torch.float32, device="cuda"),
           torch.zeros((nch, 2), dtype=torch.float32, device="cuda"))
    fr, idx, mm = K.chunk_encode_f16(_t(x), chunk, out=out)
    fr, idx, mm = _np(fr), _np(idx), _np(mm)
    for c in range(nch):
        ch = x[c * chunk:(c + 1) * chunk].astype(np.float32)
        m = O.optimal_dimensions(len(ch))[0]
        img = O.map_to_2d(ch, m)
        ridx = O.traditional_index(img, m)
        u8, mn, mx = O.normalize_u8(O.embed_index_row(img, ridx))
        assert fr[c][: m + 1, :m].tobytes() == u8.tobytes(), c
        assert idx[c][:m].tobytes() == ridx.tobytes(), c
        assert mm[c, 0] == mn and mm[c, 1] == mx


def test_pipeline_dropin_roundtrip(hq_lib):
    from hq_mi355x.api import HilbertQuantizer
    from hq_mi355x.exceptions import QuantizationError
    pytest.importorskip("PIL")
    hq = HilbertQuantizer()
    rng = np.random.default_rng(0)
    p = rng.standard_normal(1024).astype(np.float32)
    qm = hq.quantize(p, model_id="m0")
    ref_idx = O.streaming_index(O.map_from_2d(O.map_to_2d(p, 32)), 32)
    assert qm.hierarchical_indices.tobytes() == ref_idx.tobytes()
    rec = hq.reconstruct(qm)
    assert rec.shape == (1024,) and np.corrcoef(rec, p)[0, 1] > 0.9
    with pytest.raises(QuantizationError, match="Efficiency ratio 0.375 is below minimum 0.5"):
        hq.quantize(rng.standard_normal(1536).astype(np.float32))
