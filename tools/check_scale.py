"""Size-independent validity checks of a GPU-built index at large n (GPU box).

usage: python tools/check_scale.py <n_tokens> [--sa]

1. BWT symbol histogram == T' histogram.
2. (--sa) SA adjacent pairs in sorted order on a random sample (suffixes
   compared on their first 64 symbols, ties allowed only if both run past 64).
3. Every true n-gram of F (random start, length 1..8) has a non-empty range,
   and its count equals the count from a brute-force scan of the text for a
   handful of short patterns.
"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]

from fmidx.fm_index import FMIndex, suffix_sort_device  # noqa: E402
from fmidx.synth import markov_corpus_gpu  # noqa: E402

SHIFT = 10


def main():
    n_tok = int(float(sys.argv[1]))
    want_sa = "--sa" in sys.argv
    dev = torch.device("cuda", 0)
    t0 = time.time()
    text, _ = markov_corpus_gpu(n_tok, 128256, 20250905, dev)
    n = text.numel()
    bwt, sa = suffix_sort_device(text, want_sa=want_sa)
    torch.cuda.synchronize()
    print(f"n={n} built in {time.time() - t0:.1f}s", flush=True)
    h1 = torch.bincount(text, minlength=128256 + SHIFT + 1)
    h2 = torch.bincount(bwt, minlength=128256 + SHIFT + 1)
    print("histogram equal:", bool(torch.equal(h1, h2)), flush=True)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    if sa is not None:
        perm_ok = True
        k = 1 << 20
        j = torch.randint(0, n - 1, (k,), generator=g, device=dev)
        a = sa[j]
        b = sa[j + 1]
        off = torch.arange(64, device=dev)
        pa = (a[:, None] + off[None, :])
        pb = (b[:, None] + off[None, :])
        ta = torch.where(pa < n, text[pa.clamp(max=n - 1)].to(torch.int64), torch.full_like(pa, -1))
        tb = torch.where(pb < n, text[pb.clamp(max=n - 1)].to(torch.int64), torch.full_like(pb, -1))
        diff = ta != tb
        first = torch.where(diff.any(1), diff.to(torch.int8).argmax(1), torch.full_like(a, 64))
        idx = first.clamp(max=63)
        va = ta.gather(1, idx[:, None]).squeeze(1)
        vb = tb.gather(1, idx[:, None]).squeeze(1)
        ok = (first == 64) | (va < vb)
        print(f"SA sample sorted: {int(ok.sum())}/{k}; ties past 64: {int((first == 64).sum())}; "
              f"sa range ok: {bool((sa.min() >= 0).item() and (sa.max() < n).item())}", flush=True)
        perm_ok = bool(ok.all())
        del sa
    fm = FMIndex(device=0)
    fm.initialize_from_bwt_device(bwt)
    torch.cuda.synchronize()
    print("index built", fm.stats(), flush=True)
    B = 4096
    lens = torch.randint(1, 9, (B,), generator=g, device=dev)
    q = torch.randint(0, n - 20, (B,), generator=g, device=dev)
    offs = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    tot = int(offs[-1].item())
    row_of = torch.repeat_interleave(torch.arange(B, device=dev), lens)
    kk = torch.arange(tot, device=dev) - offs[:-1][row_of]
    fpos = q[row_of] + kk
    toks = text[(n - 2) - fpos].to(torch.int64) - SHIFT
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.zeros(B, dtype=torch.int64, device=dev)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    torch.cuda.synchronize()
    sent = (toks < 0).to(torch.int64)
    has_sent = torch.zeros(B, dtype=torch.int64, device=dev).index_add_(0, row_of, sent) > 0
    nonempty = (hi > lo) | has_sent
    print(f"true n-grams non-empty: {int(nonempty.sum())}/{B}", flush=True)
    bad = torch.nonzero(~nonempty).squeeze(1)[:5].tolist()
    for r in bad:
        print("  bad row", r, "len", int(lens[r]), "q", int(q[r]), "range", int(lo[r]), int(hi[r]))
    # brute-force counts of a few unigrams / bigrams over the whole text
    F = torch.flip(text[:-1], [0]).to(torch.int64) - SHIFT
    for r in range(6):
        p = toks[offs[r]:offs[r] + min(2, int(lens[r]))]
        m = torch.ones(F.numel() - p.numel() + 1, dtype=torch.bool, device=dev)
        for i in range(p.numel()):
            m &= F[i:F.numel() - p.numel() + 1 + i] == p[i]
        l2 = torch.zeros(1, dtype=torch.int64, device=dev)
        h2_ = torch.zeros(1, dtype=torch.int64, device=dev)
        fm.backward_search_batch(p.clone(), torch.tensor([0, p.numel()], device=dev), SHIFT, l2, h2_)
        print(f"  pattern {p.tolist()}: brute {int(m.sum())} index {int(h2_ - l2)}", flush=True)
    print("CHECK", "ok" if bool(nonempty.all()) else "FAIL")


if __name__ == "__main__":
    main()
