"""Oracle pinning (CPU): hand-derived known answers and the golden vectors
produced by the reference's own index.py (tests/golden/make_golden.py)."""
import itertools

import numpy as np
import pytest

from oracle.fm_oracle import NaiveFMIndex, OracleIndex, UINT64_MAX, allowed_mask, suffix_array, wm_node_count


# Hand derivation for docs [[1,2,3],[2,3,4]] ("Oracle"):
#   T' = [13,12,11,14,13,12] + sentinel 0
#   SA = [6,2,5,1,4,0,3], BWT = [12,12,13,13,14,0,11], C = {0:0,11:1,12:2,13:4,14:6}
TOY = [[1, 2, 3], [2, 3, 4]]


def test_toy_known_answers():
    idx = OracleIndex()
    idx.initialize(TOY, in_memory=True)
    assert idx.size() == 7 and len(idx) == 6 and idx.n_docs == 2
    assert idx.sa.tolist() == [6, 2, 5, 1, 4, 0, 3]
    assert idx.bwt.tolist() == [12, 12, 13, 13, 14, 0, 11]
    assert idx.get_range([2]) == (2, 4)
    assert idx.get_range([2, 3]) == (4, 6)
    assert idx.get_range([3, 4]) == (6, 7)
    assert idx.get_range([4, 1]) == (1, 2)          # n-gram across the doc boundary of F
    assert idx.get_range([3, 2]) == (0, 0)
    assert idx.get_range([5]) == (0, 0)             # unknown token
    assert idx.get_range([]) == (0, 7)
    assert idx.get_distinct_count(2, 4) == ([3], [2])
    assert idx.get_distinct_count(4, 6) == ([4], [1])   # sentinel dropped
    assert idx.distinct_count(4, 6) == (0, 1, 14, 1)
    # token 1 only occurs at BWT row n-1, which occurring_distinct excludes (index.py:67)
    assert idx.occurring_distinct == [2, 3, 4] and idx.occurring_counts == [2, 2, 1]
    assert [idx.locate(r) for r in range(8)] == [6, 2, 5, 1, 4, 0, 3, UINT64_MAX]
    assert idx.get_doc(0) == [2, 3, -10] and idx.get_doc(1) == [3, 4, 1]
    assert idx.backward_search_step(12, 0, 100) == (2, 4)   # high clamp
    assert idx.backward_search_step(12, 5, 4) == (0, 0)     # low > high
    assert idx.backward_search_step(99, 0, 6) == (0, 0)     # unknown symbol


def test_suffix_array_matches_brute_force():
    rng = np.random.default_rng(0)
    for _ in range(200):
        n = int(rng.integers(1, 60))
        k = int(rng.integers(1, 5))
        t = np.concatenate([rng.integers(1, k + 1, size=n - 1), [0]]).astype(np.int64)
        sa = suffix_array(t)
        brute = sorted(range(n), key=lambda i: t[i:].tolist())
        assert sa.tolist() == brute


def _check_case(idx, case):
    assert idx.size() == case["n"]
    assert len(idx) == case["len"]
    assert idx.beginnings == case["beginnings"]
    assert sorted(idx.occurring) == case["occurring"]
    assert idx.occurring_distinct == case["occurring_distinct"]
    assert idx.occurring_counts == case["occurring_counts"]
    assert idx.bwt.tolist() == case["bwt"]
    for p, lo, hi, cnt in case["get_range"]:
        assert idx.get_range(p) == (lo, hi), p
        assert idx.get_count(p) == cnt
    for a, b, d, c, raw, dist in case["distinct_count"]:
        assert idx.get_distinct_count(a, b) == (d, c)
        assert list(idx.distinct_count(a, b)) == raw
        assert idx.get_distinct(a, b) == dist
    multi = idx.get_distinct_count_multi(case["multi"]["lows"], case["multi"]["highs"])
    assert [[list(a), list(b)] for a, b in multi] == case["multi"]["out"]
    for s, lo, hi, out in case["backward_search_step"]:
        assert list(idx.backward_search_step(s, lo, hi)) == out
    for q, out in case["backward_search_multi"]:
        assert list(idx.backward_search_multi(q)) == out
    for r, out in case["locate"]:
        assert idx.locate(r) == out
    for a, b, out in case["extract_text"]:
        assert list(idx.extract_text(a, b)) == out
    for d, doc in case["get_doc"]:
        assert idx.get_doc(d) == doc
    for r, d in case["doc_index_from_row"]:
        assert idx.get_doc_index_from_row(r) == d


def test_oracle_matches_reference_golden(golden_index_cases):
    """OracleIndex (restated index.py) == reference index.py on the same sdsl restatement."""
    seen = 0
    for case in golden_index_cases:
        if "docs" not in case:
            continue
        idx = OracleIndex()
        idx.initialize(case["docs"], in_memory=case["in_memory"])
        _check_case(idx, case)
        seen += 1
    assert seen >= 9


def test_sample_corpus_faithful_parse_is_empty(golden_index_cases):
    case = [c for c in golden_index_cases if c["name"] == "sample_corpus_faithful_empty"][0]
    assert case["n"] == 1 and case["len"] == 0 and case["occurring_distinct"] == []
    idx = OracleIndex()
    idx.initialize([], in_memory=True)
    for p, lo, hi, cnt in case["get_range"]:
        assert idx.get_range(p) == (lo, hi)
    norm = [c for c in golden_index_cases if c["name"] == "sample_corpus_normalized"][0]
    assert norm["faithful_docs"] == 0 and norm["n_docs"] == 10


def test_allowed_mask_and_node_count_definitions():
    idx = OracleIndex()
    idx.initialize(TOY, in_memory=True)
    m = allowed_mask(idx, [0, 2, 4, 0], [7, 4, 6, 0], vocab=6)
    assert m[0].nonzero()[0].tolist() == [1, 2, 3, 4]
    assert m[1].nonzero()[0].tolist() == [3]
    assert m[2].nonzero()[0].tolist() == [4]
    assert m[3].sum() == 0
    # BWT[0:7) symbols {0,11,12,13,14}; prefixes at depth 1..4 of 4-bit codes
    assert wm_node_count(idx, 0, 7, 4) == sum(
        len({s >> (4 - d) for s in [0, 11, 12, 13, 14]}) for d in range(1, 5))


def test_extract_unbounded_case_rejected():
    idx = NaiveFMIndex()
    idx.initialize([11, 12, 13])
    with pytest.raises(ValueError):
        idx.extract_text(4, 9)


def test_get_distinct_count_multi_postprocessing(golden_index_cases):
    """fmidx.index.FMIndex.get_distinct_count_multi filters and shifts the
    batched launch's result arrays (sentinel dropped, ids - SHIFT) instead of
    walking SWIG tuples per symbol; fed the oracle's raw distinct_count output
    in the launch's layout it must give the golden multi results (index.py:161-174)."""
    import numpy as np

    from fmidx.index import FMIndex

    checked = 0
    for case in golden_index_cases:
        if "docs" not in case or not case["multi"]["lows"]:
            continue
        ora = OracleIndex()
        ora.initialize(case["docs"], in_memory=case["in_memory"])
        lows, highs = case["multi"]["lows"], case["multi"]["highs"]
        raws = [ora.distinct_count(a, b) for a, b in zip(lows, highs)]

        def arrays(lo, hi, raws=raws):
            flat = [x for r in raws for x in r]
            offs = np.concatenate([[0], np.cumsum([len(r) // 2 for r in raws])]).astype(np.uint64)
            return np.asarray(flat + [0, 0], dtype=np.uint64), offs

        idx = object.__new__(FMIndex)        # no device: only the host post-processing runs
        idx._distinct_count_multi_arrays = arrays
        multi = idx.get_distinct_count_multi(lows, highs)
        assert [[list(a), list(b)] for a, b in multi] == case["multi"]["out"], case["name"]
        checked += 1
    assert checked >= 5
