"""Round-6 hardening of the peer exchange's producer and the build options
(ADVICE r5):

  * the payload decode (fm_decode_step_payload) updating its state IN PLACE,
    captured once into a HIP graph and replayed for many steps with B > 1 --
    the flag barrier's serving form -- equals the same steps decoded with
    ping-pong state buffers, eagerly: states and payload rows, every step;
  * fm_set_build_options on an index that is already built is refused, and
    the options reported stay the ones the index was built with."""
import ctypes

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
