"""Synthetic corpora and GPU index construction for benchmarks.

* ``markov_corpus_gpu``: order-1 Markov chain whose rows are Zipf(1.1) over
  a seeded id permutation, mixed 50/50 between a global permutation
  (Zipfian unigrams) and a per-row shifted one (Markov dependence), doc
  lengths lognormal with mean ~500, encoded exactly as index.py:47-53
  (each doc reversed, ids + SHIFT, concatenated) plus the sentinel 0.
* ``suffix_array_gpu``: prefix doubling on the GPU (ranks = group-head
  positions, one 64-bit key sort per round).  Construction tooling only --
  the query path never touches it.
"""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np
import torch

SHIFT = 10
_MUL = 7919          # coprime with 128256 = 2^8 * 3 * 167


def _zipf_cdf(vocab: int, s: float, device) -> torch.Tensor:
    k = torch.arange(1, vocab + 1, dtype=torch.float64, device=device)
    p = k.pow(-s)
    c = torch.cumsum(p, 0)
    return c / c[-1]


def markov_corpus_gpu(n_tokens: int, vocab: int, seed: int, device, mean_len: float = 500.0,
                      sigma: float = 1.0, zipf_s: float = 1.1, max_len_factor: float = 8.0,
                      global_mix: float = 0.5) -> Tuple[torch.Tensor, torch.Tensor]:
    """Returns (T' with sentinel as int32 [n_tokens + 1], beginnings int64 [docs + 1])."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    mu = math.log(mean_len) - sigma * sigma / 2
    max_len = int(mean_len * max_len_factor)
    est_docs = int(n_tokens / mean_len * 1.2) + 16
    lens = torch.empty(est_docs, dtype=torch.float64, device=device).log_normal_(mu, sigma, generator=g)
    lens = lens.round().clamp_(1, max_len).to(torch.int64)
    csum = torch.cumsum(lens, 0)
    ndocs = int(torch.searchsorted(csum, torch.tensor([n_tokens], device=device)).item()) + 1
    while ndocs > lens.numel():   # pragma: no cover - extremely unlikely
        more = torch.full((est_docs,), int(mean_len), dtype=torch.int64, device=device)
        lens = torch.cat([lens, more])
        csum = torch.cumsum(lens, 0)
        ndocs = int(torch.searchsorted(csum, torch.tensor([n_tokens], device=device)).item()) + 1
    lens = lens[:ndocs].clone()
    prev_total = int(csum[ndocs - 2].item()) if ndocs > 1 else 0
    lens[-1] = n_tokens - prev_total
    beginnings = torch.zeros(ndocs + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=beginnings[1:])
    # generate docs longest-first so the active docs at step t are a prefix
    order = torch.argsort(lens, descending=True)
    lens_sorted = lens[order]
    begs_sorted = beginnings[:-1][order]
    counts = torch.bincount(lens_sorted.clamp(max=max_len + 1), minlength=max_len + 2)
    # active(t) = number of docs with len > t
    active_by_t = (lens_sorted.numel() - torch.cumsum(counts, 0)).tolist()
    cdf = _zipf_cdf(vocab, zipf_s, device)
    text = torch.empty(n_tokens + 1, dtype=torch.int32, device=device)
    text[-1] = 0
    prev = torch.randint(0, vocab, (ndocs,), generator=g, device=device, dtype=torch.int64)
    salt = int(seed) * 2654435761 % vocab
    t = 0
    L0 = int(lens_sorted[0].item())
    while t < L0:
        a = active_by_t[t] if t < len(active_by_t) else 0
        if a <= 0:
            break
        u = torch.rand(a, generator=g, device=device, dtype=torch.float64)
        rk = torch.searchsorted(cdf, u).clamp_(max=vocab - 1)
        p = prev[:a]
        # mixture: a global Zipf component (Zipfian unigrams, e.g. "the", ",")
        # and a row-specific one (order-1 Markov dependence)
        glob = torch.rand(a, generator=g, device=device) < global_mix
        off = torch.where(glob, torch.full_like(p, salt), (p * 40503 + salt) % vocab)
        tok = (rk * _MUL + off) % vocab
        prev[:a] = tok
        # forward token t of doc d lands at beginnings[d] + len[d] - 1 - t  (reversed doc)
        pos = begs_sorted[:a] + lens_sorted[:a] - 1 - t
        text[pos] = (tok + SHIFT).to(torch.int32)
        t += 1
    return text, beginnings


# "Paraphrase:" as three fixed token ids, and the eos id (Llama-3 <|end_of_text|>):
# the PAQ index's docs are tokenizer("Paraphrase: " + question) + [eos]
# (/root/reference/build_fm_index.py:46-48); the real tokenizer is not available
# offline, so the prefix is a stand-in of the same shape.
PAQ_PREFIX = (62, 1768, 25)
PAQ_EOS = 128001


def paq_corpus_gpu(n_tokens: int, vocab: int, seed: int, device, prefix=PAQ_PREFIX, eos: int = PAQ_EOS,
                   mean_question: float = 20.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """A PAQ-shaped corpus: ~24-token docs, every one
    ``prefix + question + [eos]``, the questions from the same Markov / Zipf
    chain as markov_corpus_gpu (lognormal lengths around ``mean_question``,
    sigma 0.3).  Encoded exactly as index.py:47-53 (each doc reversed, ids +
    SHIFT, concatenated) plus the sentinel.  Every doc shares the prefix, so
    the prefix pattern's range holds one row per doc (tens of millions at
    n = 1.5e9) and in F every eos is followed by the prefix of the next doc.
    Returns (T' int32 [n_tokens + 1], beginnings int64 [docs + 1])."""
    extra = len(prefix) + 1
    q_total = int(n_tokens * mean_question / (mean_question + extra))
    qtext, qbeg = markov_corpus_gpu(q_total, vocab, seed, device, mean_len=mean_question, sigma=0.3,
                                    max_len_factor=3.0)
    qtext[qtext == eos + SHIFT] = eos - 1 + SHIFT      # eos is a special token: never inside a question
    nd = qbeg.numel() - 1
    qlen = qbeg[1:] - qbeg[:-1]
    beg = torch.zeros(nd + 1, dtype=torch.int64, device=device)
    torch.cumsum(qlen + extra, 0, out=beg[1:])
    n = int(beg[-1].item())
    text = torch.empty(n + 1, dtype=torch.int32, device=device)
    text[-1] = 0
    # per doc (reversed): [eos] + reversed question (= qtext's own doc slice) + reversed prefix
    text[beg[:-1]] = eos + SHIFT
    for j, t in enumerate(reversed(prefix)):
        text[beg[1:] - len(prefix) + j] = t + SHIFT
    chunk = 1 << 27
    for a in range(0, q_total, chunk):
        b = min(q_total, a + chunk)
        pos = torch.arange(a, b, dtype=torch.int64, device=device)
        doc = torch.searchsorted(qbeg, pos, right=True) - 1
        text[pos + 1 + extra * doc] = qtext[a:b]
        del pos, doc
    return text, beg


def suffix_array_gpu(text: torch.Tensor, sym_bits: int = 17) -> torch.Tensor:
    """SA of ``text`` (int32, unique minimal sentinel last) by prefix doubling.
    Requires n < 2^31.  Returns int64 [n]."""
    n = text.numel()
    if n >= (1 << 31):
        raise ValueError("suffix_array_gpu: n must be < 2^31")
    dev = text.device
    t = text.to(torch.int64)
    # first round: 3 symbols packed into one key
    k = t << (2 * sym_bits)
    k[:-1] |= t[1:] << sym_bits
    k[:-2] |= t[2:]
    del t
    h = 3
    while True:
        keys, sa = torch.sort(k)
        del k
        head = torch.ones(n, dtype=torch.bool, device=dev)
        head[1:] = keys[1:] != keys[:-1]
        del keys
        gid = torch.cumsum(head, 0)
        ngroups = int(gid[-1].item())
        heads = torch.nonzero(head).squeeze(1)      # group-head positions
        del head
        grp = heads[gid - 1]
        del gid, heads
        rank = torch.empty_like(grp)
        rank[sa] = grp
        del grp
        if ngroups == n:
            return sa
        del sa
        k = rank << 32
        k[:-h] |= rank[h:] + 1
        del rank
        h *= 2


def bwt_from_sa(text: torch.Tensor, sa: torch.Tensor) -> torch.Tensor:
    n = text.numel()
    prev = sa - 1
    prev[prev < 0] = n - 1
    return text[prev]


def decode_trace(fm, text: torch.Tensor, bwt: torch.Tensor, B: int, V: int, S: int, seed: int, device):
    """The bench's decode trace, built on the device, untimed.

    B rows start from true corpus patterns of U{1..32} tokens (n-grams of F =
    reverse(T')); each step a live row appends a true continuation (the BWT
    symbol of a uniformly chosen row of its range: a random occurrence's next
    token) with p = 0.9, else a uniform random id; a row whose range went empty
    restarts (token -1 = empty pattern = the full range).  Row 0 is an
    empty-pattern row, row 1 an eos-terminated (empty-range) row fed an unknown
    id.  Returns (tokens [S, B], (lo0, hi0), lo_hist [S, B], hi_hist [S, B],
    patterns0): the ranges after every step come from fm.decode_step itself, and
    ``patterns0`` (host lists) are the rows' initial patterns, from which
    ``trace_patterns`` gives every row's whole pattern after any step (for the
    reference-faithful full re-search)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed + 1)
    n = bwt.numel()
    lens = torch.randint(1, 33, (B,), generator=g, device=device)
    q = torch.randint(0, n - 40, (B,), generator=g, device=device)
    offs = torch.zeros(B + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=offs[1:])
    tot = int(offs[-1].item())
    row_of = torch.repeat_interleave(torch.arange(B, device=device), lens)
    k = torch.arange(tot, device=device) - offs[:-1][row_of]
    toks = text[(n - 2) - (q[row_of] + k)].to(torch.int64) - SHIFT
    lo = torch.zeros(B, dtype=torch.int64, device=device)
    hi = torch.zeros(B, dtype=torch.int64, device=device)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    lo[0], hi[0] = 0, n          # empty-pattern row
    lo[1], hi[1] = 0, 0          # eos-terminated row
    init = (lo.clone(), hi.clone())
    tok_h = toks.cpu().tolist()
    off_h = offs.cpu().tolist()
    pats = [tok_h[off_h[b]:off_h[b + 1]] for b in range(B)]
    pats[0] = []
    pats[1].append(V + 1000)     # the eos row: an unknown id ends its pattern, as its (0, 0) state says
    return _trace_steps(fm, bwt, lo, hi, init, pats, B, V, S, g, device)


def _trace_steps(fm, bwt, lo, hi, init, pats, B, V, S, g, device):
    """The steps of a decode trace from the rows' current ranges: a live row
    appends the BWT symbol of a uniformly chosen row of its range (a random
    occurrence's next token) with p = 0.9, else a uniform random id; an empty
    row restarts (token -1); row 0 always restarts, row 1 gets an unknown id."""
    n = bwt.numel()
    tokens = torch.empty((S, B), dtype=torch.int64, device=device)
    lo_hist = torch.empty((S, B), dtype=torch.int64, device=device)
    hi_hist = torch.empty((S, B), dtype=torch.int64, device=device)
    dummy = torch.empty((1, 1), dtype=torch.uint8, device=device)
    for s in range(S):
        live = lo < hi
        width = (hi - lo).clamp(min=1)
        u = torch.rand(B, generator=g, device=device, dtype=torch.float64)
        j = (lo + (u * width.to(torch.float64)).to(torch.int64).clamp(max=n - 1)).clamp(max=n - 1)
        true_tok = bwt[j].to(torch.int64) - SHIFT
        rnd = torch.randint(0, V, (B,), generator=g, device=device)
        coin = torch.rand(B, generator=g, device=device) < 0.9
        tok = torch.where(coin & (true_tok >= 0), true_tok, rnd)
        tok = torch.where(live, tok, torch.full_like(tok, -1))
        tok[0] = -1
        tok[1] = V + 1000             # unknown id: the eos row stays empty
        tokens[s] = tok
        fm.decode_step(tok, lo, hi, dummy, 0, SHIFT, reset_below=0)
        lo_hist[s] = lo
        hi_hist[s] = hi
    torch.cuda.synchronize(device)
    return tokens, init, lo_hist, hi_hist, pats


def paq_trace(fm, text: torch.Tensor, bwt: torch.Tensor, beg: torch.Tensor, B: int, V: int, S: int, seed: int,
              device, prefix=PAQ_PREFIX):
    """The C5 decode trace on a paq_corpus_gpu index (nq_open eval shape: the
    processors search force_decoding_from + sentence, force_decoding_from being
    the docs' shared prefix): a quarter of the rows start from the prefix alone
    (one row per doc in its range), half from the prefix + the first 1..8
    question tokens of a random doc, a quarter from random true n-grams of F
    (U{1..32}, as decode_trace); then _trace_steps.  Rows 0 / 1 as decode_trace.
    Returns decode_trace's tuple."""
    g = torch.Generator(device=device)
    g.manual_seed(seed + 1)
    n = bwt.numel()
    nd = beg.numel() - 1
    P = len(prefix)
    pats = []
    kinds = torch.randint(0, 4, (B,), generator=g, device=device).tolist()
    docs = torch.randint(0, nd, (B,), generator=g, device=device)
    ks = torch.randint(1, 9, (B,), generator=g, device=device).tolist()
    ends = beg[docs + 1]        # doc d occupies T'[beg[d], beg[d+1]): the prefix is its LAST P tokens (reversed)
    q = torch.randint(0, n - 40, (B,), generator=g, device=device)
    lens = torch.randint(1, 33, (B,), generator=g, device=device).tolist()
    q_h = q.tolist()
    e_h = ends.tolist()
    dlen = (beg[docs + 1] - beg[docs]).tolist()
    for b in range(B):
        if kinds[b] == 0:
            pats.append(list(prefix))
        elif kinds[b] in (1, 2):
            # forward doc = prefix, q1, q2, ...: T'[end - 1 - j] is forward token j
            k = min(ks[b], dlen[b] - P - 1)       # within the question (the doc ends with eos)
            fwd = text[torch.arange(e_h[b] - 1, e_h[b] - 1 - (P + k), -1, device=device)].to(torch.int64) - SHIFT
            pats.append(fwd.tolist())
        else:
            idx = (n - 2) - (q_h[b] + torch.arange(lens[b], device=device))
            pats.append((text[idx].to(torch.int64) - SHIFT).tolist())
    pats[0] = []
    flat = torch.tensor([t for p in pats for t in p], dtype=torch.int64, device=device)
    offs = torch.tensor([0] + list(np.cumsum([len(p) for p in pats])), dtype=torch.int64, device=device)
    lo = torch.zeros(B, dtype=torch.int64, device=device)
    hi = torch.zeros(B, dtype=torch.int64, device=device)
    fm.backward_search_batch(flat, offs, SHIFT, lo, hi)
    lo[0], hi[0] = 0, n
    lo[1], hi[1] = 0, 0
    pats[1].append(V + 1000)
    init = (lo.clone(), hi.clone())
    return _trace_steps(fm, bwt, lo, hi, init, pats, B, V, S, g, device)


def trace_patterns(patterns0, tokens, upto: int):
    """Every row's whole pattern after step ``upto`` (inclusive) of a
    decode_trace: the initial pattern plus the appended tokens, emptied by a
    restart (token < 0)."""
    pats = [list(p) for p in patterns0]
    rows = tokens[: upto + 1].tolist() if hasattr(tokens, "tolist") else tokens[: upto + 1]
    for row in rows:
        for b, t in enumerate(row):
            if t < 0:
                pats[b] = []
            else:
                pats[b].append(int(t))
    return pats
