"""The sdsl-faithful CPU restatement (bench cpu_baseline) agrees with the
naive oracle -- both are checkers, so they are cross-checked here (CPU)."""
import numpy as np

from oracle.cpu_ref import CpuRef
from oracle.fm_oracle import OracleIndex, allowed_mask


def _corpus(seed, n_docs, vocab, max_len):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, vocab, size=int(rng.integers(1, max_len))).tolist() for _ in range(n_docs)]


def test_cpu_ref_matches_oracle():
    for seed, vocab in [(1, 7), (2, 300), (3, 128256)]:
        docs = _corpus(seed, 60, vocab, 50)
        ora = OracleIndex()
        ora.initialize(docs, in_memory=True)
        ref = CpuRef.from_bwt(ora.bwt)
        n = ora.size()
        rng = np.random.default_rng(seed)
        for _ in range(300):
            a = int(rng.integers(0, n + 1))
            b = int(rng.integers(0, n + 3))
            assert ref.distinct_count(a, b) == ora.distinct_count(a, b)
            c = int(rng.choice(ora.bwt)) if rng.random() < 0.8 else int(rng.integers(0, vocab + 20))
            assert ref.backward_search_step(c, a, b) == ora.backward_search_step(c, a, b)


def test_cpu_ref_decode_and_full_step():
    docs = _corpus(5, 80, 40, 60)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    ref = CpuRef.from_bwt(ora.bwt)
    n = ora.size()
    rng = np.random.default_rng(2)
    B, V = 12, 45
    pats = [rng.integers(0, 40, size=int(rng.integers(1, 4))).tolist() for _ in range(B)]
    lo = np.zeros(B, dtype=np.uint64)
    hi = np.zeros(B, dtype=np.uint64)
    mask = np.zeros((B, V), dtype=np.uint8)
    toks = np.array([t for p in pats for t in p], dtype=np.int64)
    offs = np.zeros(B + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(p) for p in pats])
    ref.full_step(toks, offs, 10, lo, hi, mask, 4)
    want = [ora.get_range(p) for p in pats]
    assert list(zip(lo.tolist(), hi.tolist())) == want
    assert np.array_equal(mask, allowed_mask(ora, [w[0] for w in want], [w[1] for w in want], V))
    nxt = rng.integers(-1, 40, size=B).astype(np.int64)
    ref.decode_step(nxt, 10, 0, lo, hi, mask, 3)
    exp = []
    for (l, h), t in zip(want, nxt.tolist()):
        if t < 0:
            exp.append((0, n))
        elif l >= h:
            exp.append((0, 0))
        else:
            exp.append(ora.backward_search_step(t + 10, l, h - 1))
    assert list(zip(lo.tolist(), hi.tolist())) == exp
    assert np.array_equal(mask, allowed_mask(ora, [e[0] for e in exp], [e[1] for e in exp], V))
    # the timed single-thread step (the bench's in-leg distinct_count breakdown): same results, and
    # the distinct_count time it reports is a part of its own wall time
    lo2, hi2 = np.array([w[0] for w in want], dtype=np.uint64), np.array([w[1] for w in want], dtype=np.uint64)
    mask2 = np.zeros_like(mask)
    import time
    a = time.perf_counter()
    t_dist = ref.decode_step_timed(nxt, 10, 0, lo2, hi2, mask2)
    wall = time.perf_counter() - a
    assert np.array_equal(lo2, lo) and np.array_equal(hi2, hi) and np.array_equal(mask2, mask)
    assert 0.0 < t_dist <= wall
