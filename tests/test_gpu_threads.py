"""Re-entrancy of the search drop-in (SURVEY.md §8b "Threading"): the reference calls its engines from
ThreadPoolExecutor workers (core/video_search.py:806,854; core/streaming_processor.py:294; api.py:233-297),
so one engine / one resident corpus must give every thread exactly what a serial caller gets.

8 threads share ONE ProgressiveSimilaritySearchEngine (its pool corpus, scan workspace and redo counters)
and ONE IndexCorpus, on torch's default stream (the stream every thread gets unless it picks one: their
launches interleave on it) and on a stream per thread.  Pools of 12,800 rows: random index vectors, and
64-row runs of near-duplicates whose lists end in near-ties (the longer-list retry and the dense path run
inside the threads).  Every threaded result must equal the serial run byte for byte."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RUN, NB, THREADS = 64, 200, 8


def _np(x):
    from hq_mi355x._dev import to_np
    return to_np(x)


def _indices(seed, clustered):
    """[NB * RUN, 64] f64 index vectors (the fused map + index kernel on random 1536-D embeddings) and 48
    queries; clustered: NB base vectors repeated in runs of RUN + N(0, 0.01), queries drawn from the runs."""
    import torch
    from hq_mi355x import kernels as K
    g = torch.Generator(device="cuda").manual_seed(seed)
    n = NB if clustered else NB * RUN
    _, B, _ = K.map_index_quantize(torch.randn((n, 1536), generator=g, device="cuda", dtype=torch.float32), 64, 64)
    if clustered:
        C = B.repeat_interleave(RUN, 0)
        C.add_(0.01 * torch.randn(C.shape, generator=g, device="cuda", dtype=torch.float64))
        Q = B[:48] + 0.01 * torch.randn((48, 64), generator=g, device="cuda", dtype=torch.float64)
    else:
        C = B
        Q = B[::(NB * RUN) // 48][:48] + 0.01 * torch.randn((48, 64), generator=g, device="cuda",
                                                              dtype=torch.float64)
    return _np(C), _np(Q)


def _pool(C):
    from hq_mi355x.models import ModelMetadata, QuantizedModel
    return [QuantizedModel(b"x", (64, 64), 4096, 0.8, C[i], ModelMetadata(f"m{i}", 1, 1, 1.0, "t"))
            for i in range(len(C))]


def _key(results, where):
    return [(where[id(r.model)], r.similarity_score, tuple(sorted(r.matching_indices.items())),
             r.reconstruction_error) for r in results]


def _threaded(fn, items, own_stream):
    """fn over items from THREADS workers, twice over (the second round re-uses every cached buffer)."""
    import torch

    def run(x):
        if own_stream:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                out = fn(x)
            s.synchronize()
            return out
        return fn(x)

    with ThreadPoolExecutor(THREADS) as ex:
        return list(ex.map(run, list(items) * 2))


@pytest.mark.parametrize("own_stream", [False, True])
@pytest.mark.parametrize("clustered", [False, True])
@pytest.mark.parametrize("M", [20, 100])
def test_engine_threads_equal_serial(hq_lib, M, clustered, own_stream):
    """progressive_search and brute_force_search of one shared engine from 8 threads == the serial calls."""
    from hq_mi355x.core.search_engine import ProgressiveSimilaritySearchEngine
    C, Q = _indices(11 + clustered, clustered)
    pool = _pool(C)
    where = {id(m): i for i, m in enumerate(pool)}
    eng = ProgressiveSimilaritySearchEngine(similarity_threshold=0.1, max_candidates_per_level=M)
    serial = [_key(eng.progressive_search(q, pool, 10), where) for q in Q]
    bserial = [_key(eng.brute_force_search(q, pool, 10), where) for q in Q[:16]]
    corpus = eng._pool_corpus(pool)
    corpus.reset_stats()
    got = _threaded(lambda q: _key(eng.progressive_search(q, pool, 10), where), Q, own_stream)
    assert got == serial * 2
    bgot = _threaded(lambda q: _key(eng.brute_force_search(q, pool, 10), where), Q[:16], own_stream)
    assert bgot == bserial * 2
    assert eng._pool_corpus(pool) is corpus  # one resident corpus for every thread
    st = corpus.stats
    print(f"M={M} clustered={clustered} own_stream={own_stream}: {st}")
    assert st["batches"] == 2 * len(Q)
    if clustered and M == 20:
        assert st["redo_queries"] > 0, st  # the redo path ran inside the threads


@pytest.mark.parametrize("own_stream", [False, True])
@pytest.mark.parametrize("M", [20, 100])
def test_corpus_batches_threads_equal_serial(hq_lib, M, own_stream):
    """IndexCorpus.progressive / brute_force over query batches of 16 from 8 threads on one shared clustered
    corpus (retries and dense redos inside the threads) == the serial batches."""
    import torch
    from hq_mi355x.core.search_engine import IndexCorpus
    C, Q = _indices(13, True)
    Qb = [Q[i:i + 16] for i in range(0, 48, 16)] + [Q[::3], Q[1::3]]
    corpus = IndexCorpus(C)

    def prog(q):
        return [_np(x) for x in corpus.progressive(torch.from_numpy(q).cuda(), 10, 0.1, M)]

    def brute(q):
        return [_np(x) for x in corpus.brute_force(torch.from_numpy(q).cuda(), 10)]

    serial = [prog(q) for q in Qb]
    bserial = [brute(q) for q in Qb]
    corpus.reset_stats()
    # the serial batches adapted M = 20's first list length (slack_for): back to the short list, kept short, so
    # every threaded batch takes the retry
    corpus.reset_list_lengths()
    corpus.ADAPT_LISTS = False
    got = _threaded(prog, Qb, own_stream)
    bgot = _threaded(brute, Qb, own_stream)
    for a, b in zip(got, serial * 2):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    for a, b in zip(bgot, bserial * 2):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    st = corpus.stats
    print(f"M={M} own_stream={own_stream}: {st}")
    assert st["batches"] == 2 * len(Qb)
    if M == 20:
        assert st["retry_queries"] > 0, st  # the longer-list retry ran inside the threads
