"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/hq_mi355x.h declares,
and its host-only entry points (level structure, segment layout, argument validation) agree with the
reference.  No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "hq_mi355x.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^(?:int|int64_t|size_t|const char\*)\s+(hq_[a-z0-9_]+)\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from hq_mi355x import _lib
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = declared_symbols()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    from hq_mi355x._lib import SIGNATURES
    assert set(SIGNATURES) == set(names)


def test_parse_structure_matches_reference(lib, golden):
    g = golden("search")
    got = []
    buf = (ctypes.c_int32 * 64)()
    for L in list(range(1, 130)) + [256, 1024, 4096]:
        n = lib.hq_parse_structure(L, buf, 16)
        for i in range(n):
            got.append((L, buf[4 * i], buf[4 * i + 1], buf[4 * i + 2], buf[4 * i + 3]))
    np.testing.assert_array_equal(np.array(got), g["parse_struct"])


def test_segment_layout(lib):
    assert lib.hq_seg_count(64) == 5 and lib.hq_seg_padded_len(64) == 68
    assert lib.hq_seg_count(32) == 4 and lib.hq_seg_padded_len(32) == 36
    assert lib.hq_rag_index_rows(64) == 3 and lib.hq_rag_index_rows(32) == 2
    assert lib.hq_scan_workspace_size(1000, 1_000_000, 20) > 0


def test_validation_messages_match_reference(lib):
    # core/hilbert_mapper.py:136-143 messages, returned before any device work
    from hq_mi355x import _lib
    rc = lib.hq_map_to_2d(0, None, 1, 4, 4, 3, None, None)
    assert rc == _lib.HQ_E_NOT_POW2
    assert _lib.last_error() == "Dimension must be a power of 2, got 3"
    rc = lib.hq_map_to_2d(0, None, 1, 20, 20, 4, None, None)
    assert rc == _lib.HQ_E_TOO_MANY
    assert _lib.last_error() == "Too many parameters (20) for dimensions 4x4 (16 cells)"
    rc = lib.hq_hilbert_table(6, None, None, None, None)
    assert _lib.last_error() == "Grid size must be a power of 2, got 6"
    rc = lib.hq_map_index_quantize(None, 1, 4, 4, 256, 16, None, None, None, None)
    assert rc == _lib.HQ_E_UNSUPPORTED


def test_host_dimension_logic(golden):
    from hq_mi355x.core.dimension_calculator import PowerOf4DimensionCalculator
    g = golden("quant")
    dc = PowerOf4DimensionCalculator()
    for s, n, err in zip(g["dim_sizes"], g["dim_n"], g["dim_err"]):
        assert dc.calculate_optimal_dimensions(int(s)) == (n, n)
        if err:
            with pytest.raises(ValueError) as e:
                dc.calculate_padding_strategy(int(s), (n, n))
            assert str(e.value) == str(err)


def test_host_allocation_logic(golden):
    from hq_mi355x.core.index_generator import level_allocation
    from hq_mi355x.rag.hierarchical_index_generator import HierarchicalIndexGenerator
    g = golden("index")
    assert [tuple(x) for x in g["trad_alloc_32"]] == level_allocation(32)
    assert [tuple(x) for x in g["trad_alloc_64"]] == level_allocation(64)
    gen = HierarchicalIndexGenerator()
    assert gen.calculate_optimal_granularity((64, 64))["granularity_levels"] == [8, 4, 2]
    assert gen.calculate_optimal_granularity((32, 32))["granularity_levels"] == [4, 2]
    for k in range(5):
        img = g[f"rag_img_{k}"]
        rows = g[f"rag_rows_{k}"]
        info = gen.calculate_optimal_granularity((img.shape[1], img.shape[0]))
        assert rows.shape[0] == img.shape[0] + info["index_rows_needed"]


def test_product_has_no_cpu_fallback():
    """The product package must not import the oracle or compute on the host when no GPU exists."""
    import hq_mi355x
    pkg = os.path.dirname(hq_mi355x.__file__)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("oracle/", ""), f
    import torch
    if not torch.cuda.is_available():
        from hq_mi355x import _lib
        from hq_mi355x.core import HilbertCurveMapper
        with pytest.raises(_lib.NativeLibraryError):
            HilbertCurveMapper().map_to_2d(np.arange(16, dtype=np.float32), (4, 4))


def test_validation_paths_of_batched_entries(lib):
    """Argument checks of the S7, pre-computed and stream entries return before any device work:
    empty problems are no-ops (HQ_OK), bad shapes are errors with the reference's messages."""
    from hq_mi355x import _lib
    assert lib.hq_cos_padded_k(1) == 32 and lib.hq_cos_padded_k(4096) == 4096 and lib.hq_cos_padded_k(0) == 0
    assert lib.hq_cos_padded_rows(1) == 128 and lib.hq_cos_padded_rows(250_000) == 250_112
    assert lib.hq_cos_scores_mfma(None, None, 0, None, None, 5, 64, None, None) == _lib.HQ_OK
    assert lib.hq_cos_scores_mfma(None, None, 3, None, None, 0, 64, None, None) == _lib.HQ_OK
    assert lib.hq_cos_scores_mfma(None, None, -1, None, None, 5, 64, None, None) == _lib.HQ_E_INVALID
    assert lib.hq_cos_scores_mfma(None, None, 3, None, None, 5, 64, None, None) == _lib.HQ_E_INVALID  # null
    assert lib.hq_cos_prepare(None, 4, 10, 16, None, None, None) == _lib.HQ_E_INVALID                # ld < K
    assert lib.hq_cos_prepare(None, 0, 16, 16, None, None, None) == _lib.HQ_OK
    assert lib.hq_seg_flag_rows(None, -1, None, None) == _lib.HQ_E_INVALID                           # bad N
    assert lib.hq_seg_flag_rows(None, 5, None, None) == _lib.HQ_E_INVALID                            # null
    rc = lib.hq_precomputed_index(0, 1, None, 1, 64, 10, 3, 6, 2, None, 64, None)
    assert rc == _lib.HQ_E_NOT_POW2 and _lib.last_error() == "Dimension must be a power of 2, got 3"
    assert lib.hq_precomputed_index(0, 1, None, 1, 64, 10, 256, 6, 2, None, 64, None) == _lib.HQ_E_UNSUPPORTED
    assert lib.hq_precomputed_index(0, 2, None, 1, 64, 10, 8, 6, 2, None, 64, None) == _lib.HQ_E_INVALID
    assert lib.hq_precomputed_index(0, 1, None, 1, 100, 65, 8, 6, 2, None, 64, None) == _lib.HQ_E_TOO_MANY
    assert lib.hq_precomputed_index(0, 1, None, 0, 64, 10, 8, 6, 2, None, 64, None) == _lib.HQ_OK
    assert lib.hq_chunk_encode_f16(None, 0, 1024, None, None, None, None) == _lib.HQ_OK
    assert lib.hq_chunk_encode_f16(None, 10, 0, None, None, None, None) == _lib.HQ_E_INVALID
    assert lib.hq_chunk_encode_f16(None, 10, 1024, None, None, None, None) == _lib.HQ_E_INVALID      # null


def test_search_host_keeps_f32_index_vectors():
    """Host dtype plumbing for hq_seg_prepare_src: float32 index vectors stay float32 until the
    corpus is prepared (the f32 flag), everything else is widened to f64 (no compute here)."""
    import numpy as np
    import torch
    from hq_mi355x.core import search_engine as se
    a32 = np.zeros(8, np.float32)
    assert se._is_f32(a32) and se._is_f32(torch.zeros(3, dtype=torch.float32))
    assert not se._is_f32(np.zeros(8)) and not se._is_f32([0.1, 0.2])
    assert se._idx(a32).dtype == np.float32
    assert se._idx([1, 2]).dtype == np.float64
    assert se._idx(np.zeros(3, np.float16)).dtype == np.float64
    assert np.stack([se._idx(a32), se._idx(a32)]).dtype == np.float32


def test_kernel_options_are_explicit(lib):
    """Kernel variants are selected only by hq_set_option: the default library imports no getenv (a stray
    environment variable cannot change a kernel path), options set / read back / reset, unknown names fail."""
    import subprocess
    from hq_mi355x import _lib
    syms = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    if lib.hq_diag_build() == 0:
        assert "getenv" not in syms
    assert _lib.get_option("fused_v") is None
    with _lib.option("fused_v", 5):
        assert _lib.get_option("fused_v") == 5
    assert _lib.get_option("fused_v") is None
    with pytest.raises(_lib.NativeLibraryError, match="unknown option 'no_such_knob'"):
        _lib.set_option("no_such_knob", 1)
    assert lib.hq_get_option(b"no_such_knob", None) == _lib.HQ_E_INVALID


def _scan0f_reads(chunk_len: int, n_rows: int) -> int:
    """Rows past its first that one k_scan0f wave reads for a chunk of n_rows rows (hq_search.hip k_scan0f:
    two steps of 16 rows are loaded before the loop, each body loads one more step; the loop runs three
    bodies while cs + 32 < c_end, then up to two tail bodies)."""
    loads, cs = 2, 0
    while cs + 32 < n_rows:
        loads += 3
        cs += 48
    loads += (cs < n_rows) + (cs + 16 < n_rows)
    return 16 * loads


def test_scan0f_reads_stay_inside_padded_copies(lib):
    """Deterministic guard for the round-2 fault class (prologue rows past the kPad0 padding): for every
    corpus size N = 1..70,000 and query counts 1..1000, the largest Z16 / S32 row any k_scan0f wave reads
    (chunks starting at or past N exit before loading) lies inside the padded copies."""
    g = [ctypes.c_int(), ctypes.c_int(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()]
    refs = [ctypes.byref(x) for x in g]
    worst = 0
    for Q in (1, 5, 63, 64, 65, 127, 500, 999, 1000):
        for N in range(1, 70_001):
            assert lib.hq_scan0_geometry(Q, N, *refs) == 0
            nchunks, cl, z_rows, s_rows = g[1].value, g[2].value, g[3].value, g[4].value
            assert cl % 16 == 0 and nchunks % 8 == 0 and nchunks * cl >= N
            last = (N - 1) // cl                       # last chunk that starts below N
            m = max(last * cl + _scan0f_reads(cl, N - last * cl) - 1,
                    (last - 1) * cl + _scan0f_reads(cl, cl) - 1 if last > 0 else -1)
            assert m < z_rows and m < s_rows, (Q, N, m, z_rows)
            worst = max(worst, m - N)
    assert worst == 46  # reads reach row N + 46: inside the 48 padding rows, 1 row to spare


def test_bench_traffic_table_well_formed():
    """Every kernel bench.py cites in its `traffic` field has a numeric per-launch HBM figure in the committed
    rocprofv3 PMC table (a malformed record once crashed the round-end bench)."""
    import importlib.util
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "bench.py")).read()
    names = sorted(set(re.findall(r'load_traffic\("([A-Za-z0-9_]+)"\)', src)))
    assert names
    spec = importlib.util.spec_from_file_location("_bench_mod", os.path.join(root, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    for n in names:
        v = mod.load_traffic(n)
        assert isinstance(v, float) and v > 0, (n, v)
