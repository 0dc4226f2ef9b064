"""GPU parity: the HIP engine (through libfmidx.so's C-ABI) against the oracle
and the golden vectors from the reference's own index.py.  Integer results
must be bit-exact."""
import os

import numpy as np
import pytest

from oracle.fm_oracle import NaiveFMIndex, OracleIndex, UINT64_MAX, allowed_mask

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def ours_index(docs, bm_log2=None, cache_min=None, trans=None, **options):
    """The engine index of ``docs`` built with fm_build_options fields
    (fmidx.options; small thresholds make every acceleration structure exist
    on a small corpus)."""
    from fmidx.index import FMIndex

    opts = {"bm_log2": bm_log2, "cache_min": cache_min, "transitions": trans, **options}
    idx = FMIndex(device=0, options={k: v for k, v in opts.items() if v is not None})
    idx.initialize(docs, in_memory=True)
    return idx


def markov_docs(seed, n_docs, vocab, max_len, sticky=0.7):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n_docs):
        ln = int(rng.integers(1, max_len + 1))
        tok = int(rng.integers(0, vocab))
        d = []
        for _ in range(ln):
            d.append(tok)
            tok = (tok * 31 + 7) % vocab if rng.random() < sticky else int(rng.integers(0, vocab))
        docs.append(d)
    return docs


# ---------------------------------------------------------------- golden
@pytest.mark.parametrize("gpu_sort_min", [None, 1])
def test_golden_index_cases(dev, golden_index_cases, gpu_sort_min):
    """gpu_sort_min=1: FMIndex.initialize sorts every corpus on the GPU (the
    path of corpora >= 2^20 tokens); locate / extract / get_doc go through the
    SA / ISA samples and LF walks either way."""
    from fmidx.index import FMIndex

    checked = 0
    for case in golden_index_cases:
        if "docs" not in case:
            continue
        idx = FMIndex(device=0, options={"gpu_sort_min": gpu_sort_min} if gpu_sort_min else None)
        idx.initialize(case["docs"], in_memory=case["in_memory"])
        name = case["name"]
        assert idx.size() == case["n"], name
        assert len(idx) == case["len"]
        assert idx.beginnings == case["beginnings"]
        assert sorted(idx.occurring) == case["occurring"]
        assert idx.occurring_distinct == case["occurring_distinct"], name
        assert idx.occurring_counts == case["occurring_counts"], name
        pats = [p for p, *_ in case["get_range"]]
        got = idx.get_ranges(pats)
        for (p, lo, hi, cnt), g in zip(case["get_range"], got):
            if p and min(p) + 10 < 0:
                continue
            assert g == (lo, hi), (name, p)
            assert idx.get_range(p) == (lo, hi)
            assert idx.get_count(p) == cnt
        for a, b, d, c, raw, dist in case["distinct_count"]:
            assert list(idx.distinct_count(a, b)) == raw, (name, a, b)
            assert idx.get_distinct_count(a, b) == (d, c)
            assert idx.get_distinct(a, b) == dist
        multi = idx.get_distinct_count_multi(case["multi"]["lows"], case["multi"]["highs"])
        assert [[list(a), list(b)] for a, b in multi] == case["multi"]["out"]
        for s, lo, hi, out in case["backward_search_step"]:
            assert list(idx.backward_search_step(s, lo, hi)) == out, (name, s, lo, hi)
        for q, out in case["backward_search_multi"]:
            assert list(idx.backward_search_multi(q)) == out
        for r, out in case["locate"]:
            assert idx.locate(r) == out
        for a, b, out in case["extract_text"]:
            assert list(idx.extract_text(a, b)) == out, (name, a, b)
        for d, doc in case["get_doc"]:
            assert idx.get_doc(d) == doc
        for r, d in case["doc_index_from_row"]:
            assert idx.get_doc_index_from_row(r) == d
        checked += 1
    assert checked >= 9


def test_swig_surface_errors(dev):
    from fmidx._lib import FMIndexError
    from fmidx.fm_index import FMIndex

    fm = FMIndex(device=0)
    fm.initialize([11, 12, 13, 12])
    with pytest.raises(OverflowError):
        fm.backward_search_step(-1, 0, 3)
    with pytest.raises(TypeError):
        fm.distinct_count(0.5, 3)
    with pytest.raises(FMIndexError):
        fm.extract_text(7, 9)           # unbounded loop in the reference
    with pytest.raises(FMIndexError):
        FMIndex(device=0).initialize([3, 0, 4])   # sdsl rejects a 0 symbol
    assert fm.locate(99) == UINT64_MAX


# ---------------------------------------------------------------- random corpora
@pytest.mark.parametrize("seed,n_docs,vocab,max_len,bm", [
    (1, 40, 30, 60, 6),
    (2, 200, 500, 120, 6),
    (3, 300, 128256, 80, 7),
    (4, 120, 5, 200, 5),
    (5, 400, 2000, 150, None),
    (6, 150, 1 << 20, 60, 6),     # 21-bit symbols: 3-level LF wavelet matrix
    (7, 300, 246, 90, 6),         # 8-bit symbols: one uint8 LF level
])
@pytest.mark.parametrize("cache_min", [None, 8])
def test_random_corpora_vs_oracle(dev, seed, n_docs, vocab, max_len, bm, cache_min):
    """cache_min=8: the range-bitmap cache holds every reachable range of width
    >= 8, so masks of wide ranges come from cached bitmaps."""
    import torch

    docs = markov_docs(seed, n_docs, vocab, max_len)
    ours = ours_index(docs, bm_log2=bm, cache_min=cache_min)
    if cache_min is not None and bm is not None and vocab < 10000:
        assert ours.stats()["cache_nodes"] > 1
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    assert ours.size() == n
    assert ours.occurring_distinct == ora.occurring_distinct
    assert ours.occurring_counts == ora.occurring_counts
    rng = np.random.default_rng(seed + 100)
    F = [t for d in reversed(docs) for t in d]
    pats = []
    for _ in range(300):
        s = int(rng.integers(0, len(F)))
        pats.append(F[s: s + int(rng.integers(1, 12))])
    for _ in range(100):
        pats.append([int(x) for x in rng.integers(0, vocab + 5, size=int(rng.integers(1, 4)))])
    pats.append([])
    got = ours.get_ranges(pats)
    want = [ora.get_range(p) for p in pats]
    assert got == want
    # ranges: pattern ranges + random + wide
    lows, highs = [], []
    for lo, hi in want:
        lows.append(lo)
        highs.append(hi)
    for _ in range(100):
        a = int(rng.integers(0, n + 1))
        b = int(rng.integers(a, n + 1))
        lows.append(a)
        highs.append(b)
    lows += [0, 0, n - 1, 5, 0]
    highs += [n, n - 1, n, 3, n + 9]
    assert ours.distinct_count_multi(lows, highs) == ora.distinct_count_multi(lows, highs)
    # allowed masks: unpacked and packed, token space with SHIFT
    lo_t = torch.tensor(lows, dtype=torch.int64, device=dev)
    hi_t = torch.tensor(highs, dtype=torch.int64, device=dev)
    V = min(vocab + 3, 128256)
    mask = ours.allowed_mask(lo_t, hi_t, V, 10).cpu().numpy()
    ref = allowed_mask(ora, lows, highs, V, 10)
    assert np.array_equal(mask, ref)
    packed = ours.allowed_mask(lo_t, hi_t, V, 10, packed=True).cpu().numpy().view(np.uint32)
    unpacked = np.unpackbits(packed.view(np.uint8), axis=1, bitorder="little")[:, :V]
    assert np.array_equal(unpacked, ref)
    # device distinct_count with counts
    syms, counts, k, cap_off = ours.distinct_count_batch(lo_t, hi_t)
    syms, counts, k, cap_off = [x.cpu().numpy() for x in (syms, counts, k, cap_off)]
    for i, (a, b) in enumerate(zip(lows, highs)):
        exp = ora.distinct_count(a, b)
        s0 = int(cap_off[i])
        got_i = []
        for j in range(int(k[i])):
            got_i += [int(syms[s0 + j]), int(counts[s0 + j])]
        assert tuple(got_i) == exp, (a, b)


def test_incremental_lf_equals_full_research(dev):
    """Carrying (lo, hi) across decode steps == re-running get_range on the
    whole pattern every step (index.py:103-114), including early exit."""
    import torch

    docs = markov_docs(7, 150, 60, 100)
    ours = ours_index(docs, bm_log2=6)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    F = [t for d in reversed(docs) for t in d]
    rng = np.random.default_rng(9)
    B, S = 64, 20
    starts = rng.integers(0, len(F) - S - 1, size=B)
    toks = np.zeros((S, B), dtype=np.int64)
    for b in range(B):
        for s in range(S):
            toks[s, b] = F[starts[b] + s] if rng.random() < 0.85 else int(rng.integers(0, 70))
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.full((B,), ours.size(), dtype=torch.int64, device=dev)
    for s in range(S):
        t = torch.tensor(toks[s], device=dev)
        ours.lf_step_batch(t, lo, hi, 10)
        got = list(zip(lo.cpu().tolist(), hi.cpu().tolist()))
        want = [ora.get_range(toks[: s + 1, b].tolist()) for b in range(B)]
        assert got == want, s


_GROUPED_CASES = {}


def _grouped_case(cache_min):
    """Index, oracle answers and inputs of the grouped-LF test (built once per
    cache_min and shared by every launch variant)."""
    if cache_min in _GROUPED_CASES:
        return _GROUPED_CASES[cache_min]
    docs = markov_docs(17, 400, 60, 100)
    ours = ours_index(docs, bm_log2=6, cache_min=cache_min)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ours.size()
    F = [t for d in reversed(docs) for t in d]
    rng = np.random.default_rng(23)
    m = 20011          # not a multiple of the 32 rows a two-lane wave holds
    pats = []
    for i in range(m):
        ln = int(rng.integers(0, 7))
        s = int(rng.integers(0, len(F) - ln))
        p = list(F[s:s + ln])
        for j in range(ln):
            r = rng.random()
            if r < 0.1:
                p[j] = int(rng.integers(0, 70))
            elif r < 0.12:
                p[j] = 1000 + int(rng.integers(0, 5))     # beyond the largest symbol
        pats.append(p)
    want = [ora.get_range(p) if p else (0, n) for p in pats]
    # one LF step from every pattern's range (some states past n, some reset)
    nxt = np.where(rng.random(m) < 0.8, [F[int(rng.integers(0, len(F)))] for _ in range(m)],
                   rng.integers(-3, 80, m)).astype(np.int64)
    li = [w[0] for w in want]
    hv = [w[1] for w in want]
    hv[::97] = [n + 5] * len(hv[::97])
    want_lf = []
    for i in range(m):
        t = int(nxt[i])
        if t < -2:
            want_lf.append((0, n))
        else:
            a_, b_ = li[i], min(hv[i], n)
            want_lf.append((0, 0) if a_ >= b_ else ora.backward_search_step(t + 10, a_, b_ - 1))
    _GROUPED_CASES[cache_min] = (ours, pats, want, nxt, li, hv, want_lf)
    return _GROUPED_CASES[cache_min]


# every launch variant of the LF kernels (csrc/query.hip lf_tuning): the grouped
# kernels -- lanes per row, the in-group transition probe (G >= 4), the
# four-at-a-time wide stage (G = 2) -- and the opt-in worklist sweeps
_GROUPED_VARIANTS = [{}, {"lf_group": 1}, {"lf_quad": 0}, {"lf_split": 1},
                     {"lf_split": 1, "lf_quad": 0}, {"search_group": 2},
                     {"lf_group": 4, "search_group": 4, "lf_gprobe": 0},
                     {"lf_group": 4, "search_group": 4, "lf_gprobe": 1},
                     {"lf_group": 8, "search_group": 8, "lf_gprobe": 0},
                     {"lf_group": 8, "search_group": 8, "lf_gprobe": 1},
                     {"lf_group": 16, "search_group": 16},
                     {"lf_group": 64, "search_group": 64}]
_LF_VARIANTS = _GROUPED_VARIANTS + [{"lf_work": 0}, {"lf_work": 1}, {"lf_work": 2}, {"search_p8": 0}]


@pytest.mark.parametrize("variant", _LF_VARIANTS, ids=lambda v: "-".join(f"{k}{x}" for k, x in v.items()) or "default")
@pytest.mark.parametrize("cache_min", [None, 4])
def test_grouped_lf_and_search_vs_oracle(dev, cache_min, variant):
    """Launches above lf_group_min (8192) rows take the grouped kernels
    (G lanes per row, wide rows by the whole wave): get_range of 20011
    patterns (index.py:103-114 with its early exit) and one LF step of 20011
    (state, token) pairs, against the oracle -- dead, empty, full-range,
    narrow, wide and cached rows, unknown ids, hi past n, reset rows -- for
    every launch variant (selected through fm_set_tuning in this process)."""
    import torch

    from fmidx.options import tuning

    ours, pats, want, nxt, li, hv, want_lf = _grouped_case(cache_min)
    m = len(pats)
    with tuning(**variant):
        toks = torch.tensor([t for p in pats for t in p], dtype=torch.int64, device=dev)
        offs = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pats])]), dtype=torch.int64, device=dev)
        lo = torch.zeros(m, dtype=torch.int64, device=dev)
        hi = torch.zeros(m, dtype=torch.int64, device=dev)
        ours.backward_search_batch(toks, offs, 10, lo, hi)
        got = list(zip(lo.cpu().tolist(), hi.cpu().tolist()))
        bad = [i for i in range(m) if got[i] != want[i]]
        assert not bad, [(pats[i], got[i], want[i]) for i in bad[:5]]
        lo_in = torch.tensor(li, dtype=torch.int64, device=dev)
        hi_in = torch.tensor(hv, dtype=torch.int64, device=dev)
        lo_out, hi_out = torch.empty_like(lo), torch.empty_like(hi)
        ours.lf_step_batch(torch.tensor(nxt, device=dev), lo_in, hi_in, 10, lo_out=lo_out, hi_out=hi_out,
                           reset_below=-2)
        got = list(zip(lo_out.cpu().tolist(), hi_out.cpu().tolist()))
        bad = [i for i in range(m) if got[i] != want_lf[i]]
        assert not bad, [(i, int(nxt[i]), li[i], hv[i], got[i], want_lf[i]) for i in bad[:5]]
        # in place (the decode loop's launch: outputs over the inputs)
        ours.lf_step_batch(torch.tensor(nxt, device=dev), lo_in, hi_in, 10, reset_below=-2)
        got = list(zip(lo_in.cpu().tolist(), hi_in.cpu().tolist()))
        bad = [i for i in range(m) if got[i] != want_lf[i]]
        assert not bad, [(i, int(nxt[i]), li[i], hv[i], got[i], want_lf[i]) for i in bad[:5]]


def test_lf_sweep_descents_vs_oracle(dev):
    """The in-wave LF sweep's tail rows (lf_work 2: the library's kernel from
    2^19 rows) on a corpus made for them: 17-bit symbols (a 9-bit first
    wavelet level, i.e. uint16 digits), frequent tokens whose ranges are
    wider than the sweep's E scans and narrower than the range cache (the
    descents, four per wave round), ranges ending at n with n mod 1024 in the
    block's second half (the half-block rank from the level's total), cached
    ranges with probe misses (cache_min 64), and an index without the E array
    (every row a probe or a descent) -- against the oracle."""
    import torch

    from fmidx.options import tuning

    rng = np.random.default_rng(41)

    def doc():
        ln = int(rng.integers(40, 160))
        common = rng.integers(0, 24, ln)
        rare = rng.integers(60000, 120000, ln)
        return [int(x) for x in np.where(rng.random(ln) < 0.9, common, rare)]

    docs = [doc() for _ in range(260)]
    while True:   # n mod 1024 in the second half of the last rank block
        n_est = sum(len(d) for d in docs) + 1   # T' + the sentinel
        if 600 <= n_est % 1024 <= 1000:
            break
        docs.append(doc())
    for cache_min, opts in ((None, {}), (64, {}), (None, {"lf_e": 0})):   # lf_e 0: no E array, every tail a descent
        ours = ours_index(docs, cache_min=cache_min, **opts)
        ora = OracleIndex()
        ora.initialize(docs, in_memory=True)
        n = ours.size()
        assert n == ora.size() and 600 <= n % 1024 <= 1000, n
        F = [t for d in reversed(docs) for t in d]
        m = 24001
        pats, nxt = [], []
        for i in range(m):
            ln = int(rng.integers(0, 3))
            s = int(rng.integers(0, len(F) - ln))
            pats.append(list(F[s:s + ln]))
            nxt.append(F[int(rng.integers(0, len(F)))] if rng.random() < 0.85 else int(rng.integers(0, 120000)))
        want = [ora.get_range(p) if p else (0, n) for p in pats]
        li = [w[0] for w in want]
        hv = [w[1] for w in want]
        hv[::7] = [n] * len(hv[::7])            # ranges ending at n: the last block's upper end
        li[::7] = [max(0, n - int(rng.integers(513, 4000))) for _ in range(len(li[::7]))]
        want_lf = []
        for i in range(m):
            a_, b_ = li[i], min(hv[i], n)
            want_lf.append((0, 0) if a_ >= b_ else ora.backward_search_step(int(nxt[i]) + 10, a_, b_ - 1))
        widths = np.array(hv) - np.array(li)
        assert ((widths > 512) & (widths < 4096)).sum() > 2000
        with tuning(lf_work=2):
            lo_in = torch.tensor(li, dtype=torch.int64, device=dev)
            hi_in = torch.tensor(hv, dtype=torch.int64, device=dev)
            lo_out, hi_out = torch.empty_like(lo_in), torch.empty_like(hi_in)
            ours.lf_step_batch(torch.tensor(nxt, dtype=torch.int64, device=dev), lo_in, hi_in, 10, lo_out=lo_out,
                               hi_out=hi_out, reset_below=-(1 << 62))
        got = list(zip(lo_out.cpu().tolist(), hi_out.cpu().tolist()))
        bad = [i for i in range(m) if got[i] != want_lf[i]]
        assert not bad, [(i, int(nxt[i]), li[i], hv[i], got[i], want_lf[i]) for i in bad[:5]]


def test_workspace_launches_under_graph_capture(dev):
    """The handle's workspace is never captured into a graph: an LF launch
    whose variant needs it (lf_work 1, the worklist sweep) takes the
    workspace-free kernels on a capturing stream -- the replayed graph is
    exact against the oracle -- and distinct_count_batch refuses to be
    captured (a round-5 run of a workspace launch inside a graph faulted)."""
    import torch

    from fmidx.options import tuning

    ours, pats, want, nxt, li, hv, want_lf = _grouped_case(4)
    m = len(pats)
    tok = torch.tensor(nxt, device=dev)
    lo_in = torch.tensor(li, dtype=torch.int64, device=dev)
    hi_in = torch.tensor(hv, dtype=torch.int64, device=dev)
    lo_out, hi_out = torch.zeros_like(lo_in), torch.zeros_like(hi_in)
    with tuning(lf_work=1):
        ours.lf_step_batch(tok, lo_in, hi_in, 10, lo_out=lo_out, hi_out=hi_out, reset_below=-2)   # eager: the worklist
        torch.cuda.synchronize()
        lo_out.zero_()
        hi_out.zero_()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ours.lf_step_batch(tok, lo_in, hi_in, 10, lo_out=lo_out, hi_out=hi_out, reset_below=-2)
        g.replay()
        torch.cuda.synchronize()
    got = list(zip(lo_out.cpu().tolist(), hi_out.cpu().tolist()))
    bad = [i for i in range(m) if got[i] != want_lf[i]]
    assert not bad, [(i, got[i], want_lf[i]) for i in bad[:5]]
    del g
    # the C-ABI entry itself on a capturing stream (the Python wrapper reads its capacity on the host first)
    from ctypes import c_void_p

    from fmidx._lib import last_error, lib

    lo_r = torch.tensor([1], dtype=torch.int64, device=dev)
    hi_r = torch.tensor([3], dtype=torch.int64, device=dev)
    cap_off = torch.tensor([0, 2], dtype=torch.int64, device=dev)
    syms, counts, k = (torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(3))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    rc = None
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2, stream=s):
        rc = lib().fm_distinct_count_batch(ours._h, c_void_p(lo_r.data_ptr()), c_void_p(hi_r.data_ptr()), 1,
                                           c_void_p(cap_off.data_ptr()), 2, c_void_p(syms.data_ptr()),
                                           c_void_p(counts.data_ptr()), c_void_p(k.data_ptr()), c_void_p(s.cuda_stream))
    assert rc != 0 and "not capturable" in last_error()
    torch.cuda.synchronize()
    del g2
    syms2, counts2, k2, _ = ours.distinct_count_batch(lo_r, hi_r)   # eagerly: unchanged
    assert int(k2[0].item()) >= 1


@pytest.mark.parametrize("cache_min", [None, 4])
def test_small_lf_batches_vs_oracle(dev, cache_min):
    """fm_lf_step_batch launches of <= 8192 rows (one wave per row, k_lf) --
    every row of the grouped test's 20011 (state, token) pairs (dead, empty,
    full, narrow, wide and cached ranges, unknown ids, hi past n, reset rows)
    in launches of 256 and of 37 rows, out of place and in place, against the
    oracle.  (One 1024-thread workgroup per row -- the fused kernel's LF stage
    alone, whose workgroup E scan replaces the descent of a 513..4095-row
    range -- was measured slower at C3, B = 256: 6.9 vs 6.4 us cold.)"""
    import torch

    ours, pats, want, nxt, li, hv, want_lf = _grouped_case(cache_min)
    tok_all = torch.tensor(nxt, device=dev)
    lo_all = torch.tensor(li, dtype=torch.int64, device=dev)
    hi_all = torch.tensor(hv, dtype=torch.int64, device=dev)
    M = len(nxt)
    for width in (256, 37):
        got_lo = torch.empty_like(lo_all)
        got_hi = torch.empty_like(hi_all)
        for a in range(0, M, width):
            b = min(M, a + width)
            t, l, h = tok_all[a:b].contiguous(), lo_all[a:b].clone(), hi_all[a:b].clone()
            ol, oh = torch.empty_like(l), torch.empty_like(h)
            ours.lf_step_batch(t, l, h, 10, lo_out=ol, hi_out=oh, reset_below=-2)
            ours.lf_step_batch(t, l, h, 10, reset_below=-2)   # in place
            assert torch.equal(ol, l) and torch.equal(oh, h), (width, a)
            got_lo[a:b], got_hi[a:b] = ol, oh
        got = list(zip(got_lo.cpu().tolist(), got_hi.cpu().tolist()))
        bad = [i for i in range(M) if got[i] != want_lf[i]]
        assert not bad, [(i, int(nxt[i]), li[i], hv[i], got[i], want_lf[i]) for i in bad[:5]]


@pytest.mark.parametrize("cache_min,e2", [(None, "0"), (4, "0"), (None, "1"), (4, "1")])
def test_decode_step_fused_and_reset(dev, cache_min, e2):
    """Fused LF + mask against the oracle, with and without E2 (the narrow
    rows' content read with their E scan instead of streamed afterwards)."""
    import torch

    docs = markov_docs(11, 80, 40, 90)
    ours = ours_index(docs, bm_log2=5, cache_min=cache_min, lf_e2=int(e2))
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    B, V = 16, 50
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.full((B,), n, dtype=torch.int64, device=dev)
    state = [(0, n)] * B
    rng = np.random.default_rng(3)
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    for step in range(12):
        tk = rng.integers(0, 45, size=B)
        tk[rng.random(B) < 0.2] = -1        # reset rows
        ours.decode_step(torch.tensor(tk, device=dev), lo, hi, mask, V, 10, reset_below=0)
        new = []
        for b in range(B):
            if tk[b] < 0:
                new.append((0, n))
            else:
                l, h = state[b]
                new.append((0, 0) if l >= h else ora.backward_search_step(int(tk[b]) + 10, l, h - 1))
        state = new
        assert list(zip(lo.cpu().tolist(), hi.cpu().tolist())) == state
        ref = allowed_mask(ora, [s[0] for s in state], [s[1] for s in state], V, 10)
        assert np.array_equal(mask.cpu().numpy(), ref)


@pytest.mark.parametrize("cache_min,trans,threads,V", [(None, None, None, 12), (None, 0, None, 12),
                                                       (256, None, None, 12), (64, 1, None, 12),
                                                       (600, None, None, 12), (None, None, 256, 12),
                                                       (256, None, 512, 12), (64, None, 256, 12),
                                                       (64, None, None, 151936), (64, None, 256, 151936),
                                                       (None, None, None, 128256)])
def test_decode_step_wide_ranges(dev, cache_min, trans, threads, V):
    """Decode steps through every LF path of the fused kernel: the workgroup
    E scan (uncached ranges of 513..4096 rows), the transition table (cached
    parents -> any child, incl. one-row children and cached children), the
    table restricted to cached children (trans=1), the two-level descent
    (trans=0), the wave E scan (<= 512 rows) and early zero-filled rows."""
    import torch

    docs = markov_docs(31, 400, 8, 200, sticky=0.5)     # ~40K tokens over 8 symbols
    if V > 1000:   # + rare ids over the whole vocabulary: wide ranges with allowed sets spread over V
        r2 = np.random.default_rng(7)
        docs = [[t if r2.random() < 0.7 else int(r2.integers(8, V - 10)) for t in d] for d in docs]
    ours = ours_index(docs, bm_log2=6, cache_min=cache_min, trans=trans)
    from fmidx.options import tuning

    with tuning(dec_threads=threads or 0):     # workgroup size of the decode kernel (0: by batch)
        _decode_wide_ranges(dev, ours, docs, cache_min, trans, V)


def _decode_wide_ranges(dev, ours, docs, cache_min, trans, V):
    import torch

    st = ours.stats()
    if trans != 0 and st["cache_nodes"] > 1:
        assert st["trans_entries"] > 0
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    F = [t for d in reversed(docs) for t in d]
    rng = np.random.default_rng(5)
    B, S = 96, 9
    starts = rng.integers(0, len(F) - S - 1, size=B)
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.full((B,), n, dtype=torch.int64, device=dev)
    state = [(0, n)] * B
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    seen_wg = 0
    for step in range(S):
        tk = np.array([F[starts[b] + step] if rng.random() < 0.9 else int(rng.integers(0, 10)) for b in range(B)])
        seen_wg += sum(1 for a, b in state if 512 < b - a <= 4096)
        ours.decode_step(torch.tensor(tk, device=dev), lo, hi, mask, V, 10, reset_below=0)
        new = []
        for b in range(B):
            l, h = state[b]
            new.append((0, 0) if l >= h else ora.backward_search_step(int(tk[b]) + 10, l, h - 1))
        state = new
        assert list(zip(lo.cpu().tolist(), hi.cpu().tolist())) == state, step
        ref = allowed_mask(ora, [s_[0] for s_ in state], [s_[1] for s_ in state], V, 10)
        assert np.array_equal(mask.cpu().numpy(), ref), step
    assert seen_wg > 0


def test_device_build_matches_host_build(dev):
    import torch

    from fmidx.fm_index import FMIndex

    docs = markov_docs(21, 100, 300, 100)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    bwt = torch.tensor(ora.bwt.astype(np.int32), device=dev)
    sa = torch.tensor(ora.sa.astype(np.int64), device=dev)
    text = torch.tensor(ora.text.astype(np.int32), device=dev)
    fm = FMIndex(device=0)
    fm.initialize_from_bwt_device(bwt, sa, text)
    assert fm.size() == n
    rng = np.random.default_rng(5)
    for _ in range(50):
        a = int(rng.integers(0, n))
        b = int(rng.integers(a, n + 1))
        assert fm.distinct_count(a, b) == ora.distinct_count(a, b)
        s = int(rng.integers(10, 320))
        assert fm.backward_search_step(s, a, b) == ora.backward_search_step(s, a, b)
        assert fm.locate(a) == ora.locate(a)
        if b > a:
            assert fm.extract_text(a, b) == ora.extract_text(a, b)


def test_save_load_roundtrip(dev, tmp_path):
    from fmidx.index import FMIndex

    docs = markov_docs(31, 30, 50, 40)
    a = ours_index(docs)
    a.labels = [f"doc{i}" for i in range(len(docs))]
    a.save(str(tmp_path / "idx"))
    b = FMIndex.load(str(tmp_path / "idx"), device=0)
    assert b.size() == a.size() and b.beginnings == a.beginnings and b.labels == a.labels
    assert b.occurring_distinct == a.occurring_distinct
    for d in range(len(docs)):
        assert b.get_doc(d) == a.get_doc(d)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    for r in range(b.size() + 1):             # every row from the saved SA samples, and one past the end
        assert b.locate(r) == ora.locate(r)
    assert b.get_docs(list(range(len(docs)))) == [ora.get_doc(d) for d in range(len(docs))]


def test_initialize_docs_device_path_at_scale(dev):
    """FMIndex.initialize (index.py:39-67 -> fm_initialize) of a 5e7-token
    corpus: suffix sorting on the GPU, SA / ISA samples instead of a resident
    suffix array.  locate (single and batched), get_docs and get_doc_indices
    against the full suffix array and the text."""
    import torch

    from fmidx.fm_index import suffix_sort_device
    from fmidx.index import FMIndex
    from fmidx.synth import markov_corpus_gpu

    text, beg = markov_corpus_gpu(50_000_000, 128256, 3, dev)
    T = text.cpu().numpy().astype(np.int64)
    Bg = beg.cpu().numpy()
    docs = [T[Bg[d]:Bg[d + 1]][::-1] - 10 for d in range(Bg.size - 1)]     # the forward docs
    idx = FMIndex(device=0)
    idx.initialize(docs)
    n = text.numel()
    assert idx.size() == n and idx.beginnings == Bg.tolist()
    st = idx.stats()
    assert 0 < st["sample_bytes"] < n * 2          # samples, not an 8n-byte suffix array
    _, sa = suffix_sort_device(text, want_sa=True)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    rows = torch.cat([torch.randint(0, n, (200000,), generator=g, device=dev),
                      torch.tensor([0, 1, n - 2, n - 1], device=dev)])
    assert torch.equal(idx.locate_batch(rows), sa[rows])
    assert int(idx.locate_batch(torch.tensor([n, n + 5], device=dev))[0]) == -1   # UINT64_MAX
    for r in rows[:20].tolist():
        assert idx.locate(r) == int(sa[r])
    pick = np.random.default_rng(2).choice(Bg.size - 1, size=300, replace=False).tolist() + [0, Bg.size - 2]
    for d, got in zip(pick, idx.get_docs(pick)):
        e = int(Bg[d + 1])                     # get_doc(d): T'[(end - 2 - j) mod n] - SHIFT, j < len(d)
        want = [int(T[(e - 2 - j) % n]) - 10 for j in range(len(docs[d]))]
        assert got == want, d
    assert idx.get_doc(pick[0]) == idx.get_docs(pick[:1])[0]
    F = T[:-1][::-1]
    pat = F[123456:123459].tolist()
    pat = [t - 10 for t in pat]
    lo, hi = idx.get_range(pat)
    assert hi > lo
    want = (np.searchsorted(Bg, sa[lo:hi].cpu().numpy(), side="right") - 1).tolist()
    assert list(idx.get_doc_indices(pat)) == want


def test_properties_at_scale(dev):
    """Size-independent properties on a ~1M-token index: counts sum to the
    range width, mask popcount == number of distinct symbols, LF of every
    distinct symbol has width == its count."""
    import torch

    from fmidx.index import FMIndex

    rng = np.random.default_rng(77)
    docs = [rng.integers(0, 20000, size=int(rng.integers(50, 1500))).tolist() for _ in range(1200)]
    idx = FMIndex(device=0)
    idx.initialize(docs, in_memory=True)
    n = idx.size()
    m = 64
    a = rng.integers(0, n, size=m)
    w = np.minimum(rng.integers(1, 400000, size=m), n - a)
    b = a + w
    lo_t = torch.tensor(a, dtype=torch.int64, device=dev)
    hi_t = torch.tensor(b, dtype=torch.int64, device=dev)
    syms, counts, k, off = idx.distinct_count_batch(lo_t, hi_t)
    mask = idx.allowed_mask(lo_t, hi_t, 20010, 10)
    k = k.cpu().numpy()
    off = off.cpu().numpy()
    syms = syms.cpu().numpy()
    counts = counts.cpu().numpy()
    pop = mask.sum(1).cpu().numpy()
    for i in range(m):
        s0 = off[i]
        c = counts[s0: s0 + k[i]]
        sy = syms[s0: s0 + k[i]]
        assert int(c.sum()) == int(b[i] - a[i])
        assert int(pop[i]) == int((sy >= 10).sum())
        assert np.all(np.diff(sy) > 0)
        for j in rng.choice(int(k[i]), size=min(5, int(k[i])), replace=False):
            lo2, hi2 = idx.backward_search_step(int(sy[j]), int(a[i]), int(b[i]) - 1)
            assert hi2 - lo2 == int(c[j])


def test_doc_sharded_masks_on_gpu(dev):
    """Two doc-range shards (with halo) built as separate GPU indexes: the OR
    of their masks equals the unsharded mask through incremental steps."""
    import torch

    from fmidx.index import FMIndex
    from fmidx.sharding import ShardedDecoder, shard_corpus

    docs = markov_docs(41, 120, 80, 60)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    F = [t for d in reversed(docs) for t in d]
    rng = np.random.default_rng(8)
    B, V, steps = 48, 90, 6
    starts = rng.integers(0, len(F) - 30, size=B)
    pats = [F[s: s + int(rng.integers(1, 6))] for s in starts]
    decs = []
    for r in range(3):
        sd, _ = shard_corpus(docs, 3, r, halo=5 + steps + 1)
        ix = FMIndex(device=0)
        ix.initialize(sd, in_memory=True)
        decs.append(ShardedDecoder(ix, V, 10))
    masks = [d.start(pats, dev) for d in decs]
    got = masks[0] | masks[1] | masks[2]
    want = allowed_mask(ora, *zip(*[ora.get_range(p) for p in pats]), V, 10)
    assert np.array_equal(got.cpu().numpy(), want)
    cur = [list(p) for p in pats]
    pos = [s + len(p) for s, p in zip(starts, pats)]
    for _ in range(steps):
        tk = [F[pos[b]] if rng.random() < 0.8 else int(rng.integers(0, 85)) for b in range(B)]
        pos = [p + 1 for p in pos]
        cur = [c + [t] for c, t in zip(cur, tk)]
        t = torch.tensor(tk, dtype=torch.int64, device=dev)
        ms = [d.step(t) for d in decs]
        got = ms[0] | ms[1] | ms[2]
        want = allowed_mask(ora, *zip(*[ora.get_range(c) for c in cur]), V, 10)
        assert np.array_equal(got.cpu().numpy(), want)


# ---------------------------------------------------------------- GPU construction
def _sa_cases():
    rng = np.random.default_rng(404)
    cases = {
        "single": [0],
        "two": [11, 0],
        "run": [12] * 300 + [0],                               # one symbol: log2(n) rounds
        "period3": ([11, 12, 13] * 200) + [0],
        "period7_mixed": ([14, 11, 11, 12, 15, 11, 13] * 90) + [16, 0],
        "binary_random": rng.integers(1, 3, size=2000).tolist() + [0],
        "zipfish": (np.minimum(rng.zipf(1.3, size=5000), 5000) + 10).tolist() + [0],
        "big_symbols": (rng.integers(10, 130000, size=3000)).tolist() + [0],
        "wide_symbols": (rng.integers(10, (1 << 20), size=1500)).tolist() + [0],   # 1 symbol per first key
    }
    return cases


@pytest.mark.parametrize("chunk", [None, "1024"])
def test_gpu_suffix_sort_vs_oracle(dev, chunk):
    """fm_suffix_sort_device == suffix sorting by definition, including the
    multi-chunk and larger-than-a-chunk group paths (tuning sa_chunk = 1024)."""
    import torch

    from fmidx.fm_index import suffix_sort_device
    from oracle.fm_oracle import suffix_array

    from fmidx.options import tuning

    with tuning(sa_chunk=int(chunk) if chunk else 1 << 29):
        for name, t in _sa_cases().items():
            text = np.asarray(t, dtype=np.int64)
            want = suffix_array(text)
            tt = torch.tensor(text.astype(np.int32), device=dev)
            bwt, sa = suffix_sort_device(tt, want_sa=True)
            assert np.array_equal(sa.cpu().numpy(), want), name
            n = text.size
            want_bwt = text[(want + n - 1) % n]
            assert np.array_equal(bwt.cpu().numpy(), want_bwt.astype(np.int32)), name


def test_gpu_suffix_sort_rejects_bad_sentinel(dev):
    import torch

    from fmidx import FMIndexError
    from fmidx.fm_index import suffix_sort_device

    for bad in ([11, 12, 13], [11, 0, 12, 0], [0, 11, 12]):
        with pytest.raises(FMIndexError):
            suffix_sort_device(torch.tensor(bad, dtype=torch.int32, device=dev))


def test_initialize_from_text_device_vs_oracle(dev):
    import torch

    from fmidx.fm_index import FMIndex

    docs = markov_docs(55, 200, 400, 120)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    text = torch.tensor(ora.text.astype(np.int32), device=dev)
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text, keep_sa_text=True)
    n = ora.size()
    assert fm.size() == n
    rng = np.random.default_rng(9)
    for _ in range(100):
        a = int(rng.integers(0, n))
        b = int(rng.integers(a, n + 1))
        s = int(rng.integers(10, 420))
        assert fm.backward_search_step(s, a, b) == ora.backward_search_step(s, a, b)
        assert fm.distinct_count(a, b) == ora.distinct_count(a, b)
        assert fm.locate(a) == ora.locate(a)


def test_wt_int_levels_device(dev):
    import torch

    from fmidx.fm_index import wt_int_levels_device
    from oracle.cpu_ref import levels_numpy

    rng = np.random.default_rng(3)
    for n, hi in ((1, 2), (63, 40), (64, 300), (1000, 130000), (4099, 17)):
        b = rng.integers(0, hi, size=n).astype(np.int64)
        L = max(1, int(b.max()).bit_length())
        got = wt_int_levels_device(torch.tensor(b.astype(np.int32), device=dev), L).cpu().numpy().view(np.uint64)
        assert np.array_equal(got, levels_numpy(b, L)), (n, hi)


def test_gpu_suffix_sort_at_scale_matches_doubling(dev):
    """~50M-token synthetic corpus: the chunked GPU sorter and the torch
    prefix-doubling builder agree on the whole BWT (forced small chunks)."""
    import torch

    from fmidx.fm_index import suffix_sort_device
    from fmidx.synth import bwt_from_sa, markov_corpus_gpu, suffix_array_gpu

    text, _ = markov_corpus_gpu(50_000_000, 128256, 99, dev)
    want = bwt_from_sa(text, suffix_array_gpu(text))
    from fmidx.options import tuning

    with tuning(sa_chunk=1 << 22):
        got, _ = suffix_sort_device(text)
    assert torch.equal(got, want)


def test_distinct_workspace_across_streams(dev):
    """fm_distinct_count_batch on a side stream and the host-API
    distinct_count_multi (internal stream) share the k_distinct workspace;
    interleaved, every result must still equal the oracle's."""
    import torch

    docs = markov_docs(61, 300, 3000, 150)
    ours = ours_index(docs)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    rng = np.random.default_rng(17)
    side = torch.cuda.Stream(device=dev)
    for it in range(6):
        a = rng.integers(0, n, size=200)
        b = np.minimum(a + rng.integers(1, 5000, size=200), n)
        lo_t = torch.tensor(a, dtype=torch.int64, device=dev)
        hi_t = torch.tensor(b, dtype=torch.int64, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            res = ours.distinct_count_batch(lo_t, hi_t)
        a2 = rng.integers(0, n, size=50).tolist()
        b2 = [min(x + int(rng.integers(1, 20000)), n) for x in a2]
        assert ours.distinct_count_multi(a2, b2) == ora.distinct_count_multi(a2, b2)
        side.synchronize()
        syms, counts, k, cap_off = [x.cpu().numpy() for x in res]
        for i in range(0, 200, 7):
            s0 = int(cap_off[i])
            got = []
            for j in range(int(k[i])):
                got += [int(syms[s0 + j]), int(counts[s0 + j])]
            assert tuple(got) == ora.distinct_count(int(a[i]), int(b[i])), (it, i)


def test_sharded_decode_at_scale_one_gpu(dev):
    """Doc-range sharding at 1e8 tokens on one GPU, in process: three shards
    built on the device (shard_text_device: one slice of T' each), every row
    decoded against every shard into bit-packed rows, ORed by fm_or_bits --
    equal, step by step, to the unsharded index's uint8 masks.  The same
    shards through ShardedDecoder (uint8 rows, OR on the host side of the
    test) agree too."""
    import torch

    from fmidx.fm_index import FMIndex, suffix_sort_device
    from fmidx.sharding import ShardedDecoder, or_bits, shard_text_device
    from fmidx.synth import decode_trace, markov_corpus_gpu

    V, B, S, H = 128256, 64, 6, 64
    text, beg = markov_corpus_gpu(100_000_000, V, 13, dev)
    bwt, _ = suffix_sort_device(text)
    full = FMIndex(device=0)
    full.initialize_from_bwt_device(bwt)
    tokens, init, lo_hist, hi_hist, pats0 = decode_trace(full, text, bwt, B, V, S, 99, dev)
    del bwt
    assert max(len(p) for p in pats0) + S <= H - 1
    shards = []
    for r in range(3):
        t_r, _ = shard_text_device(text, beg, 3, r, H)
        ix = FMIndex(device=0)
        ix.initialize_from_text_device(t_r)
        shards.append(ix)
    decs = [ShardedDecoder(ix, V, 10, halo=H) for ix in shards]
    starts = [d.start(pats0, dev) for d in decs]
    want0 = full.allowed_mask(init[0], init[1], V, 10)
    assert torch.equal(starts[0] | starts[1] | starts[2], want0)
    Wd = (V + 31) // 32
    st = []
    for ix in shards:
        lo = torch.zeros(B, dtype=torch.int64, device=dev)
        hi = torch.zeros(B, dtype=torch.int64, device=dev)
        offs = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pats0])]), device=dev)
        toks = torch.tensor([t for p in pats0 for t in p], dtype=torch.int64, device=dev)
        ix.backward_search_batch(toks, offs, 10, lo, hi)
        st.append((lo, hi))
    parts = torch.empty((3, B, Wd), dtype=torch.int32, device=dev)
    for s in range(S):
        for r, ix in enumerate(shards):
            lo2, hi2 = torch.empty_like(st[r][0]), torch.empty_like(st[r][1])
            ix.decode_step(tokens[s], st[r][0], st[r][1], parts[r], V, 10, reset_below=0, lo_out=lo2, hi_out=hi2,
                           packed=True)
            st[r] = (lo2, hi2)
        got = or_bits(parts, V)
        want = full.allowed_mask(lo_hist[s], hi_hist[s], V, 10)
        assert torch.equal(got, want), s
        ms = [d.step(tokens[s]) for d in decs]
        assert torch.equal(ms[0] | ms[1] | ms[2], want), s
    packed_or = or_bits(parts, V, unpack=False)
    assert torch.equal(packed_or, parts[0] | parts[1] | parts[2])


def test_distinct_count_batch_capacity_overflow(dev):
    """fm_distinct_count_batch's contract (include/fmidx.h): a row whose distinct
    symbols exceed its capacity reports k = UINT64_MAX and writes nothing --
    for a BFS row, a cached row (k_distinct_cached) and the full range; the rows
    around it, with enough capacity, are exact."""
    import torch

    docs = markov_docs(71, 300, 40, 120)
    ours = ours_index(docs, bm_log2=5, cache_min=4)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    n = ora.size()
    assert ours.stats()["trans_entries"] > 0
    F = [t for d in reversed(docs) for t in d]
    cand = [ora.get_range(F[s:s + 1]) for s in range(0, 400, 7)]
    cached = [r for r in cand if r[1] - r[0] >= 8 and
              bool(ours.cache_contains(torch.tensor([r[0]], device=dev), torch.tensor([r[1]], device=dev))[0])]
    uncached = [(a, a + 40) for a in range(3, n - 50, 997)]
    assert cached, "no cached range among the unigram ranges"
    rows = [cached[0], (0, n), uncached[0], cached[-1], (0, n), uncached[-1]]
    lo = torch.tensor([r[0] for r in rows], dtype=torch.int64, device=dev)
    hi = torch.tensor([r[1] for r in rows], dtype=torch.int64, device=dev)
    ks = [len(ora.distinct_count(a, b)) // 2 for a, b in rows]
    assert all(k >= 2 for k in ks[:3])
    cap = torch.tensor([1, 1, 1, ks[3], ks[4], ks[5]], dtype=torch.int64, device=dev)   # first three too small
    syms, counts, k, cap_off = ours.distinct_count_batch(lo, hi, cap=cap)
    syms, counts, k, cap_off = [x.cpu().numpy() for x in (syms, counts, k, cap_off)]
    assert k[:3].tolist() == [-1, -1, -1]
    for i in range(3, 6):
        a, b = rows[i]
        s0 = int(cap_off[i])
        got = []
        for j in range(int(k[i])):
            got += [int(syms[s0 + j]), int(counts[s0 + j])]
        assert tuple(got) == ora.distinct_count(a, b), i


def _device_u8(ptr, nbytes, owner):
    """A uint8 torch view of nbytes of device memory at ptr (kept alive by owner)."""
    import torch

    class _V:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2,
                                    "strides": None}

        def __init__(self):
            self.owner = owner

    return torch.as_tensor(_V(), device=torch.device("cuda", 0))


def test_device_structs(dev):
    """fm_device_struct (the bench's gather ceilings over the index's own
    allocations) reports each structure's pointer and size, and the structures
    are what the kernels assume: E[i] = LF(i) | BWT[i] << 36 with LF the
    stable order of the BWT by symbol (LF(i) = C[BWT[i]] + rank), and the
    transition table is 8-slot buckets of 16-B slots (trans_key,
    csrc/fmidx_internal.h), each filled from its first slot, whose entries are
    children LF_c(P): a range inside c's C-block, with a one-row child's only
    symbol or a cached child's bitmap (exactly its symbols) beside it."""
    import torch

    docs = markov_docs(11, 300, 200, 120)
    ours = ours_index(docs, bm_log2=5, cache_min=4)
    n = ours.size()
    p0, b0 = ours.device_struct(0)
    # the plain BWT is freed once E holds the symbols: fm_device_struct reports none, and
    # fm_device_bwt materialises the symbols from E
    assert p0 == 0 and b0 == 0 and ours.stats()["bwt_bytes"] == 0
    bwt = ours.device_bwt().to(torch.int64)
    p1, b1 = ours.device_struct(1)
    assert p1 and b1 == 8 * n
    E = _device_u8(p1, b1, ours).view(torch.int64)
    assert torch.equal(E >> 36, bwt)
    lf = E & ((1 << 36) - 1)
    order = torch.argsort(bwt, stable=True)
    assert torch.equal(lf[order], torch.arange(n, device=dev))
    p2, b2 = ours.device_struct(2)
    assert p2 and b2 > 0 and b2 % 128 == 0
    tab = _device_u8(p2, b2, ours).view(torch.int64).cpu().numpy().view(np.uint64).reshape(-1, 8, 2)
    empty = tab[:, :, 0] == np.uint64(2**64 - 1)
    assert not (empty[:, :-1] & ~empty[:, 1:]).any()          # filled from the first slot
    st = ours.stats()
    assert int((~empty).sum()) == st["trans_entries"] > 0
    bw = bwt.cpu().numpy()
    C = np.concatenate([[0], np.cumsum(np.bincount(bw))])
    p3, b3 = ours.device_struct(3)
    bm_words = b3 // (4 * st["cache_nodes"])
    bm = _device_u8(p3, b3, ours).view(torch.int32).cpu().numpy().view(np.uint32).reshape(-1, bm_words)
    kinds = [0, 0, 0]
    for b, k in zip(*np.nonzero(~empty)):
        w0, w1 = int(tab[b, k, 0]), int(tab[b, k, 1])
        pid, c, kind = w0 & (2**20 - 1), (w0 >> 20) & (2**18 - 1), (w0 >> 38) & 3
        clo = (w0 >> 40) | ((w1 & 0x3FF) << 24)
        cw, aux = (w1 >> 10) & (2**34 - 1), w1 >> 44
        assert pid < st["cache_nodes"] and cw > 0
        assert C[c] <= clo and clo + cw <= C[c + 1]            # LF_c(P) lies in c's C-block
        kinds[kind] += 1
        if kind == 1:
            assert cw == 1 and aux == bw[clo]
        elif kind == 2:
            syms = np.unique(bw[clo:clo + cw])
            syms = syms[syms < 32 * bm_words]
            bits = np.unpackbits(bm[aux].view(np.uint8), bitorder="little")
            assert np.array_equal(np.nonzero(bits)[0], syms)
    assert kinds[2] > 0
    for w in (3, 4):
        p, b = ours.device_struct(w)
        assert p and b > 0
    with pytest.raises(Exception):
        ours.device_struct(9)
