"""Mask and range parity at BASELINE.json's full sizes, on the GPU.

* C3 shape: n = 4.4e9 > 2^32 rows (64-bit positions), decode steps at B = 256
  (1024-thread decode geometry) and at C5's B = 2048 (256-thread geometry).
* C2 shape: n = 3e8, B = 32.

Every step's ranges AND full [B, 128256] masks are compared with the
sdsl-faithful CPU restatement (oracle/cpu_ref.cpp, an independent wt_int +
rank_support_v implementation) fed the same tokens; 1- and 2-token patterns are
also checked against a brute-force scan of the text ("the tokens that follow
every occurrence").  Reference semantics: fm_index.cpp:67-97 (LF step),
:119-144 (distinct symbols), index.py:103-114 (get_range), and the boolean
core of document_constrained_generation_causal_qwen.py:189-204.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHIFT = 10
V = 128256


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _build(n_tokens, seed, dev):
    import torch

    from fmidx.fm_index import FMIndex
    from fmidx.synth import markov_corpus_gpu

    torch.cuda.empty_cache()   # blocks torch cached for earlier tests: the index is hipMalloc'd beside them
    text, beg = markov_corpus_gpu(n_tokens, V, seed, dev)
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text, keep_sa_text=True)     # GPU sort, SA / ISA samples, index
    torch.cuda.synchronize()
    return fm, text, fm.device_bwt(), beg


@pytest.fixture(scope="module")
def c3(dev):
    import torch

    if torch.cuda.get_device_properties(0).total_memory < (200 << 30):
        pytest.skip("needs a 288 GB MI355X")
    from oracle.cpu_ref import CpuRef

    fm, text, bwt, beg = _build(4_400_000_000, 7, dev)
    assert bwt.numel() > (1 << 32)
    ref = CpuRef.from_device_bwt(bwt)
    yield {"fm": fm, "text": text, "bwt": bwt, "ref": ref, "beg": beg}
    del fm, text, bwt, ref
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c2(dev):
    import torch

    from oracle.cpu_ref import CpuRef

    fm, text, bwt, beg = _build(300_000_000, 5, dev)
    ref = CpuRef.from_device_bwt(bwt)
    yield {"fm": fm, "text": text, "bwt": bwt, "ref": ref, "beg": beg}
    del fm, text, bwt, ref
    torch.cuda.empty_cache()


def _decode_vs_cpu_ref(ix, B, S, seed, dev, threads=None, monkeypatch=None):
    """S fused decode steps (LF + uint8 mask) for B rows of the bench's trace;
    every step's ranges and masks against cpu_ref fed the same tokens."""
    import torch

    from fmidx.synth import decode_trace

    from fmidx.options import tuning

    with tuning(dec_threads=threads or 0):
        return _decode_vs_cpu_ref_body(ix, B, S, seed, dev)


def _decode_vs_cpu_ref_body(ix, B, S, seed, dev):
    import torch

    from fmidx.synth import decode_trace

    fm, text, bwt, ref = ix["fm"], ix["text"], ix["bwt"], ix["ref"]
    tokens, init, _, _, _ = decode_trace(fm, text, bwt, B, V, S, seed, dev)
    lo, hi = init[0].clone(), init[1].clone()
    clo = init[0].cpu().numpy().astype(np.uint64)
    chi = init[1].cpu().numpy().astype(np.uint64)
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    cmask = np.zeros((B, V), dtype=np.uint8)
    tok_np = tokens.cpu().numpy()
    widths = []
    for s in range(S):
        fm.decode_step(tokens[s], lo, hi, mask, V, SHIFT, reset_below=0)
        ref.decode_step(np.ascontiguousarray(tok_np[s]), SHIFT, 0, clo, chi, cmask, 16)
        glo = lo.cpu().numpy().astype(np.uint64)
        ghi = hi.cpu().numpy().astype(np.uint64)
        assert np.array_equal(glo, clo) and np.array_equal(ghi, chi), f"step {s}: ranges differ"
        gm = mask.cpu().numpy()
        bad = np.nonzero((gm != cmask).any(1))[0]
        assert bad.size == 0, f"step {s}: masks differ on rows {bad[:8].tolist()}"
        widths.append(ghi.astype(np.int64) - glo.astype(np.int64))
    w = np.concatenate(widths)
    return w


@pytest.mark.timeout(900)
def test_c3_decode_b256_vs_cpu_ref(dev, c3):
    """C3 shape (n > 2^32, B = 256): the headline bench configuration."""
    w = _decode_vs_cpu_ref(c3, 256, 6, 101, dev)
    # the trace covers every row class: empty, narrow, wide, the full range
    assert (w == 0).any() and ((w > 0) & (w <= 512)).any() and (w > 4096).any()


@pytest.mark.timeout(900)
def test_c3_decode_b2048_vs_cpu_ref(dev, c3):
    """C5's row count (512 x beam 4 = 2048) on the > 2^32 index: the decode
    kernel's 256-thread geometry (several rows per CU)."""
    w = _decode_vs_cpu_ref(c3, 2048, 3, 202, dev)
    assert ((w > 512) & (w <= 4096)).any()


def _follow_scan(body, a, b=None, chunk=1 << 28):
    """Brute force over the text, in chunks (no index): the occurrences of
    [a] -- or of [a, b] -- in F and the set of tokens that follow them.  In T'
    coordinates (index.py:47-53) an occurrence of [a] at T'[j] (j >= 1) is
    followed in F by T'[j - 1]; of [a, b] at T'[j] = b, T'[j + 1] = a; an
    occurrence at j = 0 is followed by the sentinel (filtered)."""
    import torch

    n1 = body.numel()
    seen = torch.zeros(V + SHIFT, dtype=torch.bool, device=body.device)
    count = 0
    for j0 in range(0, n1, chunk):
        j1 = min(n1, j0 + chunk)
        x = body[j0:j1]
        hit = x == (a if b is None else b)
        if b is not None:
            nxt = body[j0 + 1:j1 + 1]
            hit[: nxt.numel()] &= nxt == a
            if nxt.numel() < hit.numel():
                hit[nxt.numel():] = False
        count += int(hit.sum())
        if j0 == 0:
            hit[0] = False          # followed by the sentinel
        if j0 > 0:
            prev = body[j0 - 1:j1 - 1]
        else:
            prev = torch.cat([body[:1], body[: j1 - 1]])
        seen[prev[hit].to(torch.int64)] = True
    want = seen[SHIFT:].cpu().numpy().astype(np.uint8)
    return count, want


@pytest.mark.timeout(900)
def test_c3_ngrams_vs_brute_force(dev, c3):
    """1- and 2-token patterns: the allowed set == the tokens that follow
    every occurrence in F, found by scanning the text (no index involved)."""
    import torch

    fm, text = c3["fm"], c3["text"]
    n = text.numel()
    body = text[:-1]
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    pos = torch.randint(1, n - 3, (6,), generator=g, device=dev)
    picks = body[pos].tolist()
    pats = []
    for j, a in enumerate(picks):
        pats.append([a - SHIFT])
        if j < 4:   # a true bigram of F: a, then the token after that occurrence (T'[pos - 1])
            pats.append([a - SHIFT, int(body[pos[j] - 1]) - SHIFT])
    pats.append([int(torch.argmax(torch.bincount(body[: 1 << 24], minlength=V + SHIFT))) - SHIFT])  # most frequent
    m = len(pats)
    offs = torch.tensor(np.concatenate([[0], np.cumsum([len(p) for p in pats])]), device=dev)
    toks = torch.tensor([t for p in pats for t in p], dtype=torch.int64, device=dev)
    lo = torch.zeros(m, dtype=torch.int64, device=dev)
    hi = torch.zeros(m, dtype=torch.int64, device=dev)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    got = fm.allowed_mask(lo, hi, V, SHIFT).cpu().numpy()
    for i, p in enumerate(pats):
        cnt, want = _follow_scan(body, p[0] + SHIFT, None if len(p) == 1 else p[1] + SHIFT)
        assert int(hi[i] - lo[i]) == cnt, (p, int(hi[i] - lo[i]), cnt)
        assert np.array_equal(got[i], want), p
    # the fused decode step from the full range gives the 1-gram masks too
    one = [i for i, p in enumerate(pats) if len(p) == 1]
    B = len(one)
    lo1 = torch.zeros(B, dtype=torch.int64, device=dev)
    hi1 = torch.full((B,), n, dtype=torch.int64, device=dev)
    mk = torch.empty((B, V), dtype=torch.uint8, device=dev)
    fm.decode_step(torch.tensor([pats[i][0] for i in one], device=dev), lo1, hi1, mk, V, SHIFT)
    assert np.array_equal(mk.cpu().numpy(), got[one])


@pytest.mark.timeout(900)
def test_c3_index_properties(dev, c3):
    """BWT histogram == text histogram, every true n-gram of F (B = 2048, both
    ends of the 64-bit position space) has a non-empty range."""
    import torch

    fm, text, bwt = c3["fm"], c3["text"], c3["bwt"]
    n = text.numel()
    assert torch.equal(torch.bincount(text, minlength=V + 100), torch.bincount(bwt, minlength=V + 100))
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    B = 2048
    lens = torch.randint(1, 9, (B,), generator=g, device=dev)
    q = torch.randint(0, n - 20, (B,), generator=g, device=dev)
    q[: B // 2] = q[: B // 2] % (1 << 31)
    offs = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    row_of = torch.repeat_interleave(torch.arange(B, device=dev), lens)
    k = torch.arange(int(offs[-1]), device=dev) - offs[:-1][row_of]
    toks = text[(n - 2) - (q[row_of] + k)].to(torch.int64) - SHIFT
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.zeros(B, dtype=torch.int64, device=dev)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    assert bool((hi > lo).all()), int((hi <= lo).sum())


@pytest.mark.timeout(900)
def test_c3_grouped_lf_and_search(dev, c3):
    """Above 8192 rows LF / get_range launches take the grouped kernels (G
    lanes per row).  On the > 2^32 index: get_range of 16384 true patterns
    (U{1..32} tokens) == the same patterns in two launches of 8192 (one wave
    per row); one LF step over 3 x 16384 trace pairs == the fused decode
    kernel's ranges, and a sample of 512 pairs == cpu_ref."""
    import torch

    from fmidx.synth import decode_trace

    fm, text, bwt, ref = c3["fm"], c3["text"], c3["bwt"], c3["ref"]
    n = text.numel()
    g = torch.Generator(device=dev)
    g.manual_seed(31)
    P = 16384
    lens = torch.randint(1, 33, (P,), generator=g, device=dev)
    q = torch.randint(0, n - 40, (P,), generator=g, device=dev)
    offs = torch.zeros(P + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    row_of = torch.repeat_interleave(torch.arange(P, device=dev), lens)
    k = torch.arange(int(offs[-1]), device=dev) - offs[:-1][row_of]
    toks = text[(n - 2) - (q[row_of] + k)].to(torch.int64) - SHIFT
    toks[::53] = torch.randint(0, V, toks[::53].shape, generator=g, device=dev)   # some patterns go empty
    lo = torch.zeros(P, dtype=torch.int64, device=dev)
    hi = torch.zeros(P, dtype=torch.int64, device=dev)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    lo2, hi2 = torch.zeros_like(lo), torch.zeros_like(hi)
    for a in (0, P // 2):
        o = offs[a:a + P // 2 + 1]
        t = toks[int(o[0]):int(o[-1])]
        l_, h_ = torch.zeros(P // 2, dtype=torch.int64, device=dev), torch.zeros(P // 2, dtype=torch.int64, device=dev)
        fm.backward_search_batch(t, (o - o[0]).contiguous(), SHIFT, l_, h_)
        lo2[a:a + P // 2], hi2[a:a + P // 2] = l_, h_
    assert torch.equal(lo, lo2) and torch.equal(hi, hi2)
    assert bool((hi > lo).any()) and bool((hi == 0).any())
    B, S = 16384, 4
    tokens, _, lo_h, hi_h, _ = decode_trace(fm, text, bwt, B, V, S, 515, dev)
    t = tokens[1:S].reshape(-1).contiguous()
    pl = lo_h[:S - 1].reshape(-1).contiguous()
    ph = hi_h[:S - 1].reshape(-1).contiguous()
    ol, oh = torch.empty_like(pl), torch.empty_like(ph)
    fm.lf_step_batch(t, pl, ph, SHIFT, lo_out=ol, hi_out=oh, reset_below=0)
    assert torch.equal(ol, lo_h[1:S].reshape(-1)) and torch.equal(oh, hi_h[1:S].reshape(-1))
    # the in-wave sweep (the library's choice from 2^19 rows: packed tail E scans, paired
    # descents with the two-sided block rank) on the same pairs, in place
    from fmidx.options import tuning

    with tuning(lf_work=2):
        sl, sh_ = pl.clone(), ph.clone()
        fm.lf_step_batch(t, sl, sh_, SHIFT, reset_below=0)
    assert torch.equal(sl, lo_h[1:S].reshape(-1)) and torch.equal(sh_, hi_h[1:S].reshape(-1))
    sel = torch.randint(0, t.numel(), (512,), generator=g, device=dev)
    clo = pl[sel].cpu().numpy().astype(np.uint64)
    chi = ph[sel].cpu().numpy().astype(np.uint64)
    cm = np.zeros((512, 8), dtype=np.uint8)
    ref.decode_step(np.ascontiguousarray(t[sel].cpu().numpy()), SHIFT, 0, clo, chi, cm, 16)   # ranges (+ 8 mask columns)
    assert np.array_equal(clo, ol[sel].cpu().numpy().astype(np.uint64))
    assert np.array_equal(chi, oh[sel].cpu().numpy().astype(np.uint64))
    widths = (ph - pl).cpu().numpy()
    assert (widths > 4096).any() and ((widths > 0) & (widths <= 64)).any()


@pytest.mark.timeout(600)
def test_c2_decode_b32_vs_cpu_ref(dev, c2):
    """C2 shape (simplewiki scale n = 3e8, B = 32), 12 steps."""
    w = _decode_vs_cpu_ref(c2, 32, 12, 303, dev)
    assert (w > 0).any()


@pytest.mark.timeout(600)
def test_c2_full_research_equals_incremental(dev, c2):
    """The reference re-searches the whole pattern every step (A3 x3,
    index.py:103-114); the engine carries (lo, hi).  After 20 steps the ranges
    of a full device re-search of every row's whole pattern, and cpu_ref's
    full re-search, equal the incremental state."""
    import torch

    from fmidx.synth import decode_trace, trace_patterns

    fm, text, bwt, ref = c2["fm"], c2["text"], c2["bwt"], c2["ref"]
    B, S = 32, 20
    tokens, _, lo_hist, hi_hist, pats0 = decode_trace(fm, text, bwt, B, V, S, 404, dev)
    pats = trace_patterns(pats0, tokens.cpu().numpy(), S - 1)
    lo, hi = fm.get_range_batch(pats, SHIFT)
    assert np.array_equal(lo.astype(np.int64), lo_hist[-1].cpu().numpy())
    assert np.array_equal(hi.astype(np.int64), hi_hist[-1].cpu().numpy())
    toks = np.asarray([t for p in pats for t in p], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum([len(p) for p in pats])]).astype(np.int64)
    clo = np.zeros(B, dtype=np.uint64)
    chi = np.zeros(B, dtype=np.uint64)
    cm = np.zeros((B, V), dtype=np.uint8)
    ref.full_step(toks, offs, SHIFT, clo, chi, cm, 8, faithful=True)
    # the reference's early exit maps an empty pattern range to (0, 0); the
    # empty pattern itself is (0, n)
    assert np.array_equal(clo, lo) and np.array_equal(chi, hi)
    gm = fm.allowed_mask(lo_hist[-1], hi_hist[-1], V, SHIFT).cpu().numpy()
    assert np.array_equal(gm, cm)
    del torch


@pytest.mark.timeout(900)
def test_c3_locate_extract_from_samples(dev, c3):
    """locate / extract_text on the C3 index from SA / ISA samples (no resident
    suffix array), checked through properties of the text: BWT[r] = T'[SA[r] - 1]
    for random rows (and every row of a pattern's range, whose text must spell
    the reversed pattern); get_doc (index.py:69-80) of random docs equals the
    text slice the reference's LF walk emits."""
    import torch

    fm, text, bwt, beg = c3["fm"], c3["text"], c3["bwt"], c3["beg"]
    n = text.numel()
    st = fm.stats()
    assert 0 < st["sample_bytes"] < n // 2
    g = torch.Generator(device=dev)
    g.manual_seed(21)
    rows = torch.randint(0, n, (1 << 20,), generator=g, device=dev)
    pos = fm.locate_batch(rows)
    assert bool(((pos >= 0) & (pos < n)).all())
    prev = torch.where(pos > 0, pos - 1, torch.full_like(pos, n - 1))
    assert torch.equal(text[prev], bwt[rows])
    # a pattern's occurrences: the text at every located position spells reverse(pattern)
    pat = (text[(n - 2) - (123456789 + torch.arange(4, device=dev))].to(torch.int64) - SHIFT).tolist()
    lo = torch.zeros(1, dtype=torch.int64, device=dev)
    hi = torch.zeros(1, dtype=torch.int64, device=dev)
    fm.backward_search_batch(torch.tensor(pat, device=dev), torch.tensor([0, 4], device=dev), SHIFT, lo, hi)
    r = torch.arange(int(lo), int(hi), device=dev)
    p = fm.locate_batch(r)
    for j, t in enumerate(reversed(pat)):
        assert bool((text[p + j] == t + SHIFT).all()), j
    # extract_text through the ISA samples: get_doc(d) = T'[(end - 2 - j) mod n] - SHIFT
    begs = beg.cpu().tolist()
    docs = [int(d) for d in torch.randint(0, len(begs) - 1, (64,), generator=g, device=dev).tolist()] + [0]
    b = [begs[d] for d in docs]
    e = [begs[d + 1] for d in docs]
    got = fm.extract_batch(b, e)
    for d, x, y, out in zip(docs, b, e, got):
        idx = (torch.arange(y - x, device=dev) * -1 + (y - 2)) % n
        assert list(out) == text[idx].tolist(), d
    assert fm.extract_text(b[0], e[0]) == got[0]
    assert fm.locate(int(rows[0])) == int(pos[0])


@pytest.mark.timeout(900)
@pytest.mark.parametrize("variant,B,Vs,beams", [("qwen", 256, 151936, 4), ("seq", 256, 128256, 4),
                                                ("causal", 2048, 128256, 4)])
def test_c3_processors_device_vs_host_vs_cpu_ref(dev, c3, variant, B, Vs, beams):
    """The processors on the C3 index (n > 2^32, where the range-bitmap cache,
    the transition table and the hierarchy serve k_prep's LF steps and the
    packed mask): 12 generation steps with beam reordering, the device path
    (fm_processor_call) == the host path of the same class, bit for bit; and
    every row the device path gave allowed bits has bits == the mask cpu_ref
    computes from that row's pattern, and its range == cpu_ref's get_range.
    Reference: document_constrained_generation_causal_qwen.py:101-214 (B = 256,
    Qwen3 vocabulary), document_constrained_generation_seq.py:35-123 (B = 256),
    document_constrained_generation_causal.py:74-180 (B = 2048, C5's rows)."""
    import torch

    import fmidx.processors as P

    ix, text, ref = c3["fm"], c3["text"], c3["ref"]
    n = text.numel()
    if not hasattr(ix, "occurring_distinct"):
        # the all-unigrams set of index.py:67 (A7: the full range minus BWT row n - 1, sentinel dropped)
        raw = ix.distinct_count(0, n - 1)
        ix.occurring_distinct = [s - SHIFT for s in raw[0::2] if s > 0]
    g = torch.Generator(device=dev)
    g.manual_seed({"qwen": 61, "seq": 62, "causal": 63}[variant])
    q = torch.randint(0, n - 200, (B,), generator=g, device=dev).cpu().numpy()

    def F(j):   # F = reverse(T') (index.py:47-53) token j, as a corpus token id
        return int(text[n - 2 - j]) - SHIFT

    rng = np.random.default_rng(7)
    sents = [[F(int(q[b]))] for b in range(B)]
    kw = dict(num_beams=beams, pad_token_id=0, eos_token_id=2)
    if variant == "qwen":
        mk = lambda: P.QwenIndexBasedLogitsProcessor(index=ix, min_new_tokens=3, **kw)   # noqa: E731
        head = [11, 12, 151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]
    elif variant == "causal":
        mk = lambda: P.CausalIndexBasedLogitsProcessor(index=ix, model_name="llama-3", **kw)   # noqa: E731
        head = [11, 12, 78191, 128007, 271]
    else:
        mk = lambda: P.SeqIndexBasedLogitsProcessor(index=ix, **kw)   # noqa: E731
        head = [1]                                                     # the decoder start token
    dev_p, host_p = mk(), mk()
    host_p._dev = None
    groups = B // beams
    flagged_total = 0
    for step in range(12):
        perm = np.concatenate([gr * beams + rng.permutation(beams) for gr in range(groups)])
        sents = [list(sents[i]) for i in perm]
        q = q[perm]
        if step:
            for b in range(B):
                r = rng.random()
                sents[b].append(F(int(q[b]) + len(sents[b])) if r < 0.85 else int(rng.integers(3, 128000)))
        ids = torch.tensor([head + s for s in sents], dtype=torch.int64, device=dev)
        scores = torch.randn((B, Vs), generator=g, device=dev).to(torch.bfloat16)
        want = host_p(ids, scores.clone())
        got = dev_p(ids, scores.clone())
        assert torch.equal(got.view(torch.int16), want.view(torch.int16)), (variant, step)
        bufs = dev_p._dev._bufs
        rows = np.frombuffer(bufs["rows"].cpu().numpy().tobytes(), dtype=P.ROW_DTYPE)
        fl = np.nonzero(rows["flags"] & P.FLAG_BITS)[0]
        if fl.size == 0:
            continue
        flagged_total += fl.size
        pats = [sents[i] for i in fl]
        toks = np.asarray([t for p in pats for t in p], dtype=np.int64)
        offs = np.concatenate([[0], np.cumsum([len(p) for p in pats])]).astype(np.int64)
        clo = np.zeros(fl.size, dtype=np.uint64)
        chi = np.zeros(fl.size, dtype=np.uint64)
        cm = np.zeros((fl.size, Vs), dtype=np.uint8)
        ref.full_step(toks, offs, SHIFT, clo, chi, cm, 16)
        mlo = bufs["mlo"].cpu().numpy().astype(np.uint64)[fl]
        mhi = bufs["mhi"].cpu().numpy().astype(np.uint64)[fl]
        assert np.array_equal(mlo, clo) and np.array_equal(mhi, chi), (variant, step)
        bits = bufs["bits"][torch.tensor(fl, device=dev)].cpu().numpy()
        unpacked = np.unpackbits(bits.view(np.uint8), axis=1, bitorder="little")[:, :Vs]
        bad = np.nonzero((unpacked != cm).any(1))[0]
        assert bad.size == 0, (variant, step, fl[bad[:8]].tolist())
    assert flagged_total > B          # most rows took the allowed-bits path
    assert dev_p._dev.prev_ids is not None


@pytest.mark.timeout(900)
def test_c2_bwt_equals_host_sais(dev, c2, monkeypatch):
    """The whole BWT of the C2-scale corpus (n = 3e8) from the GPU suffix
    sorter (prefix doubling, csrc/sa.hip -- the index of the c2 fixture) ==
    the BWT from the host SA-IS sorter (csrc/sais.h, induced sorting: no code
    shared with the GPU path), taken through the reference's own construction
    entry point FMIndex.initialize (fm_index.cpp:33-41) with the GPU sort
    switched off (the gpu_sort_min build option above n).  The host build's SA samples
    come from the host suffix array, so locate of 2^20 random rows must agree
    as well.  A heartbeat line every 30 s keeps the run visibly alive."""
    import threading
    import time

    import torch

    from fmidx.fm_index import FMIndex

    text, bwt_gpu = c2["text"], c2["bwt"]
    n = text.numel()
    body = text[:-1].to(torch.int64).cpu().numpy().astype(np.uint64)
    host = FMIndex(device=0, options={"gpu_sort_min": 1 << 40})
    err = []

    def run():
        try:
            host.initialize(body)
        except Exception as e:     # surfaced below
            err.append(e)

    th = threading.Thread(target=run)
    t0 = time.time()
    th.start()
    while th.is_alive():
        th.join(30)
        if th.is_alive():
            print(f"[host SA-IS build of n={n}: {time.time() - t0:.0f}s]", flush=True)
    assert not err, err
    print(f"host SA-IS build {time.time() - t0:.1f}s", flush=True)
    del body
    assert host.size() == n
    assert torch.equal(host.device_bwt(), bwt_gpu)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    rows = torch.randint(0, n, (1 << 20,), generator=g, device=dev)
    assert torch.equal(host.locate_batch(rows), c2["fm"].locate_batch(rows))
