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
