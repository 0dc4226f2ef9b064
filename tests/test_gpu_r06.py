"""Round-6 hardening of the peer exchange's producer and the build options
(ADVICE r5):

  * the payload decode (fm_decode_step_payload) updating its state IN PLACE,
    captured once into a HIP graph and replayed for many steps with B > 1 --
    the flag barrier's serving form -- equals the same steps decoded with
    ping-pong state buffers, eagerly: states and payload rows, every step;
  * fm_set_build_options on an index that is already built is refused, and
    the options reported stay the ones the index was built with;
  * round-6 kernels: the static split emit, the persistent LF sweep, and the
    absent-symbol probe shortcut (kProbeComplete), each against the oracle."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def test_inplace_payload_decode_replayed_equals_pingpong(dev):
    import torch

    from fmidx.index import FMIndex
    from fmidx.sharding import or_payloads, payload_capacity

    rng = np.random.default_rng(606)
    V, B, steps = 3000, 256, 40
    docs = [rng.integers(0, 2500, size=int(rng.integers(5, 500))).tolist() for _ in range(600)]
    for d in docs[::3]:
        d[:4] = [1, 2, 3, 4]
    F = [t for d in reversed(docs) for t in d]
    ix = FMIndex()
    ix.initialize(docs, in_memory=True)
    starts = rng.integers(0, len(F) - steps - 8, B)
    pats = [[]] + [[1]] + [F[s:s + int(rng.integers(1, 4))] for s in starts[2:]]
    lo, hi = ix.get_range_batch(pats, 10)
    lo0 = torch.tensor(lo.astype(np.int64), device=dev)
    hi0 = torch.tensor(hi.astype(np.int64), device=dev)
    toks = []
    plen = [len(p) for p in pats]
    for k in range(steps):
        row = []
        for b in range(B):
            p = int(starts[b]) + plen[b]
            if k % 9 == 4 and b % 5 == 0:
                t = -1                              # a restart: the row goes wide (dense payload rows)
            else:
                t = F[p] if p < len(F) and rng.random() < 0.85 else int(rng.integers(0, 2600))
            plen[b] = 0 if t < 0 else plen[b] + 1
            row.append(t)
        toks.append(torch.tensor(row, dtype=torch.int64, device=dev))
    cap = payload_capacity(B, V)

    # eager, ping-pong state buffers
    a_lo, a_hi = lo0.clone(), hi0.clone()
    b_lo, b_hi = torch.empty_like(a_lo), torch.empty_like(a_hi)
    pay_e = torch.zeros(cap, dtype=torch.int32, device=dev)
    want = []
    for k in range(steps):
        ix.decode_step_payload(toks[k], a_lo, a_hi, b_lo, b_hi, pay_e, V, 10, reset_below=0)
        a_lo, b_lo, a_hi, b_hi = b_lo, a_lo, b_hi, a_hi
        want.append((a_lo.clone(), a_hi.clone(), or_payloads(pay_e.unsqueeze(0).clone(), B, V, 10)))

    # in place, one captured step replayed for every step
    lo_g, hi_g = lo0.clone(), hi0.clone()
    pay_g = torch.zeros(cap, dtype=torch.int32, device=dev)
    tok_g = torch.empty_like(toks[0])
    tok_g.copy_(toks[0])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ix.decode_step_payload(tok_g, lo_g, hi_g, lo_g, hi_g, pay_g, V, 10, reset_below=0)
    # capture does not run the step: replay from the initial state
    lo_g.copy_(lo0)
    hi_g.copy_(hi0)
    bad = []
    for k in range(steps):
        tok_g.copy_(toks[k])
        g.replay()
        got = or_payloads(pay_g.unsqueeze(0).clone(), B, V, 10)
        if not (torch.equal(lo_g, want[k][0]) and torch.equal(hi_g, want[k][1]) and torch.equal(got, want[k][2])):
            bad.append(k)
    torch.cuda.synchronize()
    assert not bad, f"in-place replayed steps differ from ping-pong at {bad}"
    # the trace exercised every row kind: wide (after a restart), empty and narrow rows
    kinds = set()
    for a, b, _ in want:
        w = (torch.clamp(b, max=ix.size()) - a).clamp(min=0)
        kinds |= {"empty"} if int((w == 0).sum()) else set()
        kinds |= {"dense"} if int((w >= (V + 31) // 32).sum()) else set()
        kinds |= {"narrow"} if int(((w > 0) & (w < 8)).sum()) else set()
    assert kinds == {"empty", "dense", "narrow"}, kinds


def test_build_options_refused_once_built(dev):
    from fmidx._lib import lib
    from fmidx.fm_index import FMIndex
    from fmidx.options import build_options

    ix = FMIndex(device=0, options={"cache_min": 8})
    ix.initialize([10, 11, 12, 10, 11, 13, 10, 12])
    before = ix.build_options()
    o = build_options("compact")
    assert lib().fm_set_build_options(ix._h, ctypes.byref(o)) == -1
    assert b"already built" in lib().fm_last_error()
    assert ix.build_options() == before and before["cache_min"] == 8


@pytest.mark.parametrize("B", [256, 160])
def test_decode_split_emit_vs_oracle(dev, B):
    """The fused uint8 decode step at the headline's geometry (B <= 256: one
    1024-thread workgroup per row, one vocabulary slice, V = 128256) -- and,
    in a library built with FMIDX_DEC_SPLIT=1, the static split of the wide
    rows' emit (a row entering with a restart, the full range or >= cache_min
    rows emitted as two halves, the upper one by a helper workgroup; measured
    slower and off by default, profiles/r06_split/).  Every step's mask and
    state equal the oracle's, over rows that restart, stay wide (cached,
    cache_min 8), go narrow, go empty, with tokens in both halves of the
    vocabulary."""
    import torch

    from fmidx.index import FMIndex
    from oracle.fm_oracle import OracleIndex, allowed_mask

    rng = np.random.default_rng(B)
    V = 128256
    low = rng.integers(0, 400, size=120)
    high = rng.integers(64000, 128200, size=400)
    docs = []
    for _ in range(500):
        ln = int(rng.integers(10, 200))
        d = [int(low[rng.integers(0, low.size)]) if rng.random() < 0.6 else int(high[rng.integers(0, high.size)])
             for _ in range(ln)]
        docs.append(d)
    for d in docs[::4]:
        d[:3] = [7, 8, 9]                 # a shared phrase: wide ranges
    F = [t for d in reversed(docs) for t in d]
    ours = FMIndex(device=0, options={"cache_min": 8, "bm_log2": 5})
    ours.initialize(docs, in_memory=True)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    starts = rng.integers(0, len(F) - 20, B)
    pats = [[]] + [[7]] + [[7, 8]] + [F[s:s + int(rng.integers(1, 3))] for s in starts[3:]]
    lo, hi = ours.get_range_batch(pats, 10)
    lo_t = torch.tensor(lo.astype(np.int64), device=dev)
    hi_t = torch.tensor(hi.astype(np.int64), device=dev)
    lo2, hi2 = torch.empty_like(lo_t), torch.empty_like(hi_t)
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    plen = [len(p) for p in pats]
    wide_seen = 0
    for step in range(6):
        tok = []
        for b in range(B):
            p = int(starts[b]) + plen[b]
            if (b + step) % 17 == 3:
                t = -1
            elif rng.random() < 0.8 and p < len(F):
                t = F[p]
            else:
                t = int(rng.integers(0, 128200))
            tok.append(t)
            pats[b] = [] if t < 0 else pats[b] + [t]
            plen[b] = 0 if t < 0 else plen[b] + 1
        w_in = (torch.clamp(hi_t, max=ours.size()) - lo_t).clamp(min=0)
        wide_seen += int((w_in >= 8).sum())
        tk = torch.tensor(tok, dtype=torch.int64, device=dev)
        ours.decode_step(tk, lo_t, hi_t, mask, V, 10, reset_below=0, lo_out=lo2, hi_out=hi2)
        lo_t, lo2, hi_t, hi2 = lo2, lo_t, hi2, hi_t
        want = [ora.get_range(p) if p else (0, ours.size()) for p in pats]
        want = [(a, b) if b > a else (0, 0) for a, b in want]
        got = list(zip(lo_t.cpu().tolist(), hi_t.cpu().tolist()))
        # an empty pattern's range (a restart) is the full range [0, n)
        assert [(a, b) if b > a else (0, 0) for a, b in got] == want, step
        ref = allowed_mask(ora, [w[0] for w in want], [w[1] for w in want], V, 10)
        assert np.array_equal(mask.cpu().numpy(), ref), step
    assert wide_seen > 50     # the split path ran (rows entering wide)


def test_lf_persist_vs_oracle(dev):
    """The persistent LF sweep (tuning lf_work 4: heads of static 64-row
    chunks, tail rows appended to 16 shared queues and drained four at a time
    by whichever wave is free) against the oracle, on a corpus made for tail
    rows (17-bit symbols, ranges wider than the sweep's E scans and narrower
    than the range cache, ranges ending at n, cached ranges with probe misses,
    an index without E): three launches in a row (the counter sets and tags
    alternate by epoch), one of them in place; no launch gave up a wait."""
    import torch

    from fmidx._lib import lib
    from fmidx.index import FMIndex
    from fmidx.options import tuning
    from oracle.fm_oracle import OracleIndex

    rng = np.random.default_rng(43)

    def doc():
        ln = int(rng.integers(40, 160))
        common = rng.integers(0, 24, ln)
        rare = rng.integers(60000, 120000, ln)
        return [int(x) for x in np.where(rng.random(ln) < 0.9, common, rare)]

    docs = [doc() for _ in range(300)]
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    F = [t for d in reversed(docs) for t in d]
    for opts in ({}, {"cache_min": 64}, {"lf_e": 0}):
        ours = FMIndex(device=0, options=opts or None)
        ours.initialize(docs, in_memory=True)
        n = ours.size()
        for rep in range(3):
            m = 30011 + 977 * rep
            pats, nxt = [], []
            for i in range(m):
                ln = int(rng.integers(0, 3))
                s = int(rng.integers(0, len(F) - ln))
                pats.append(list(F[s:s + ln]))
                nxt.append(F[int(rng.integers(0, len(F)))] if rng.random() < 0.85 else int(rng.integers(-1, 120000)))
            want = [ora.get_range(p) if p else (0, n) for p in pats]
            li = [w[0] for w in want]
            hv = [w[1] for w in want]
            hv[::7] = [n] * len(hv[::7])
            li[::7] = [max(0, n - int(rng.integers(513, 4000))) for _ in range(len(li[::7]))]
            want_lf = []
            for i in range(m):
                a_, b_ = li[i], min(hv[i], n)
                if nxt[i] < 0:
                    want_lf.append((0, n))                     # reset_below = 0: a restart
                else:
                    want_lf.append((0, 0) if a_ >= b_ else ora.backward_search_step(int(nxt[i]) + 10, a_, b_ - 1))
            lo_in = torch.tensor(li, dtype=torch.int64, device=dev)
            hi_in = torch.tensor(hv, dtype=torch.int64, device=dev)
            tok = torch.tensor(nxt, dtype=torch.int64, device=dev)
            with tuning(lf_work=4, lf_sweep_min=1):
                if rep == 1:      # in place
                    ours.lf_step_batch(tok, lo_in, hi_in, 10, reset_below=0)
                    lo_out, hi_out = lo_in, hi_in
                else:
                    lo_out, hi_out = torch.empty_like(lo_in), torch.empty_like(hi_in)
                    ours.lf_step_batch(tok, lo_in, hi_in, 10, lo_out=lo_out, hi_out=hi_out, reset_below=0)
            got = list(zip(lo_out.cpu().tolist(), hi_out.cpu().tolist()))
            bad = [i for i in range(m) if got[i] != tuple(want_lf[i])]
            assert not bad, (opts, rep, [(i, nxt[i], li[i], hv[i], got[i], want_lf[i]) for i in bad[:5]])
        err = ctypes.c_uint32(7)
        assert lib().fm_lf_persist_status(ours._h, ctypes.byref(err)) == 0 and err.value == 0, opts


def test_probe_complete_absent_vs_oracle(dev):
    """The absent-symbol probe shortcut (kProbeComplete, fmidx_internal.h): with
    a transition table that holds every child of every cached parent, a probe
    finding no key beside a free slot ends the LF step as the empty range.  An
    index built with FMIDX_PROBE_COMPLETE=0 (the parent's bitmap word decides
    instead), the default one and one built with trans_min = 2 (an incomplete
    table: the flag stays off) all equal the oracle -- decode steps (uint8
    mask + state) and the in-wave LF sweep -- on cached parents stepped with
    symbols they lack, symbols they hold, and past-vocabulary ids."""
    import torch

    from fmidx.index import FMIndex
    from fmidx.options import tuning
    from oracle.fm_oracle import OracleIndex, allowed_mask

    rng = np.random.default_rng(61)
    V = 128256
    common = rng.choice(40, 20, replace=False)
    docs = []
    for _ in range(600):
        ln = int(rng.integers(20, 120))
        docs.append([int(common[rng.integers(0, 20)]) if rng.random() < 0.85 else int(rng.integers(0, V))
                     for _ in range(ln)])
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    F = [t for d in reversed(docs) for t in d]
    # patterns of 0-2 common tokens: wide parents (cached at cache_min 4; single tokens ~2400
    # rows, past the decode kernel's E scans, so the decode step probes them)
    B = 256
    pats = [[]] + [[int(x) for x in rng.choice(common, int(rng.integers(1, 3)))] for _ in range(B - 1)]
    want0 = [ora.get_range(p) if p else (0, len(F) + 1) for p in pats]
    completes = []
    # (flag off, on, and a table built without the one-occurrence children: incomplete, so off)
    for pc, extra in (("0", {}), ("1", {}), ("1", {"trans_min": 2})):
        old = os.environ.get("FMIDX_PROBE_COMPLETE")
        os.environ["FMIDX_PROBE_COMPLETE"] = pc
        try:
            ours = FMIndex(device=0, options={"cache_min": 4, **extra})
            ours.initialize(docs, in_memory=True)
        finally:
            if old is None:
                os.environ.pop("FMIDX_PROBE_COMPLETE")
            else:
                os.environ["FMIDX_PROBE_COMPLETE"] = old
        st = ours.stats()
        completes.append(st["trans_complete"])
        n = ours.size()
        lo, hi = ours.get_range_batch(pats, 10)
        assert [(int(a), int(b)) for a, b in zip(lo, hi)][1:] == [tuple(w) for w in want0][1:]
        # tokens: 50 % a symbol the parent lacks (a random id), 35 % a common token, 15 % past the vocabulary
        r = rng.random(B)
        tok = np.where(r < 0.5, rng.integers(0, V, B), np.where(r < 0.85, rng.choice(common, B), V + 5))
        want = []
        for b in range(B):
            a_, b_ = (0, n) if not pats[b] else want0[b]
            t = int(tok[b])
            want.append((0, 0) if a_ >= b_ else ora.backward_search_step(t + 10, a_, b_ - 1))
        want = [(a, b) if b > a else (0, 0) for a, b in want]
        lo_t = torch.tensor(np.asarray(lo, dtype=np.int64), device=dev)
        hi_t = torch.tensor(np.asarray(hi, dtype=np.int64), device=dev)
        lo_t[0], hi_t[0] = 0, n
        tk = torch.tensor(tok.astype(np.int64), device=dev)
        # the in-wave LF sweep
        lo2, hi2 = torch.empty_like(lo_t), torch.empty_like(hi_t)
        with tuning(lf_work=-1, lf_sweep_min=1):
            ours.lf_step_batch(tk, lo_t, hi_t, 10, lo_out=lo2, hi_out=hi2, reset_below=-1)
        got = [(a, b) if b > a else (0, 0) for a, b in zip(lo2.cpu().tolist(), hi2.cpu().tolist())]
        assert got == want, (pc, [(i, tok[i], want0[i], got[i], want[i]) for i in range(B) if got[i] != want[i]][:5])
        # the fused decode step
        mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
        lo3, hi3 = torch.empty_like(lo_t), torch.empty_like(hi_t)
        ours.decode_step(tk, lo_t, hi_t, mask, V, 10, reset_below=-1, lo_out=lo3, hi_out=hi3)
        got = [(a, b) if b > a else (0, 0) for a, b in zip(lo3.cpu().tolist(), hi3.cpu().tolist())]
        assert got == want, pc
        ref = allowed_mask(ora, [w[0] for w in want], [w[1] for w in want], V, 10)
        assert np.array_equal(mask.cpu().numpy(), ref), pc
        absent_wide = sum(1 for b in range(B) if want[b] == (0, 0) and want0[b][1] - want0[b][0] >= 4)
        assert absent_wide > 50, absent_wide
    assert completes == [0, 1, 0]
