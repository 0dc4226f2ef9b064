"""Doc-range sharding (fmidx.sharding) on CPU with torch.distributed/gloo,
world_size 2: OR of per-shard masks == the unsharded mask, for the initial
pattern search and for incremental decode steps (with restarts).  Each
rank's shard index is the oracle behind the FMIndex batched API (test
infrastructure); the sharding logic and the collective are the product's."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle.fm_oracle import OracleIndex, allowed_mask

V = 90
SHIFT = 10


class OracleShard:
    """Oracle index exposing the batched API ShardedDecoder uses."""

    def __init__(self, docs):
        self.ix = OracleIndex()
        self.ix.initialize(docs, in_memory=True)

    def get_range_batch(self, patterns, shift):
        assert shift == SHIFT
        r = [self.ix.get_range(p) for p in patterns]
        return np.array([a for a, _ in r], dtype=np.uint64), np.array([b for _, b in r], dtype=np.uint64)

    def lf_step_batch(self, tokens, lo, hi, shift, reset_below=-(1 << 63)):
        n = self.ix.size()
        for i in range(lo.numel()):
            t, l, h = int(tokens[i]), int(lo[i]), int(hi[i])
            if t < reset_below:
                l, h = 0, n
            elif l >= h or t + shift < 0:
                l, h = 0, 0
            else:
                l, h = self.ix.backward_search_step(t + shift, l, h - 1)
            lo[i], hi[i] = l, h
        return lo, hi

    def allowed_mask(self, lo, hi, vocab, shift):
        return torch.from_numpy(allowed_mask(self.ix, lo.tolist(), hi.tolist(), vocab, shift))


class OracleShardFused(OracleShard):
    """... plus the fused decode_step (uint8 or int32 bit-packed mask), so the
    ShardedDecoder's one-launch path and its packed all_gather run on CPU."""

    def decode_step(self, tokens, lo, hi, mask, vocab, shift, reset_below=-(1 << 63), packed=False,
                    lo_out=None, hi_out=None):
        if lo_out is None:
            lo_out, hi_out = lo, hi
        else:
            lo_out.copy_(lo)
            hi_out.copy_(hi)
        self.lf_step_batch(tokens, lo_out, hi_out, shift, reset_below)
        m = self.allowed_mask(lo_out, hi_out, vocab, shift).numpy()
        if packed:
            a = np.pad(m, ((0, 0), (0, mask.shape[1] * 32 - vocab)))
            mask.copy_(torch.from_numpy(np.packbits(a, axis=1, bitorder="little").view(np.int32).copy()))
        else:
            mask.copy_(torch.from_numpy(m))
        return mask

    def shard_pack(self, lo, hi, bits, vocab, payload=None):
        from fmidx.sharding import pack_payload_host

        return pack_payload_host(lo.numpy(), hi.numpy(), self.ix._bwt, bits.numpy(), vocab)


def make_case(seed=5):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(40):
        ln = int(rng.integers(1, 30))
        tok = int(rng.integers(0, 60))
        d = []
        for _ in range(ln):
            d.append(tok)
            tok = (tok * 17 + 3) % 60 if rng.random() < 0.7 else int(rng.integers(0, 60))
        docs.append(d)
    F = [t for d in reversed(docs) for t in d]
    B = 24
    starts = rng.integers(0, len(F) - 40, size=B)
    lens = rng.integers(1, 8, size=B)
    patterns = [F[s: s + ln] for s, ln in zip(starts, lens)]
    steps = []
    pos = [s + ln for s, ln in zip(starts, lens)]
    for _ in range(8):
        tk = []
        for b in range(B):
            r = rng.random()
            if r < 0.75:
                tk.append(F[pos[b]])
            elif r < 0.9:
                tk.append(int(rng.integers(0, 70)))
            else:
                tk.append(-1)   # restart
            pos[b] += 1
        steps.append(tk)
    return docs, patterns, steps


def expected_masks(docs, patterns, steps):
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    pats = [list(p) for p in patterns]
    out = []
    rng = [ora.get_range(p) for p in pats]
    out.append(allowed_mask(ora, [r[0] for r in rng], [r[1] for r in rng], V, SHIFT))
    for tk in steps:
        for b, t in enumerate(tk):
            pats[b] = [] if t < 0 else pats[b] + [t]
        rng = [ora.get_range(p) for p in pats]
        out.append(allowed_mask(ora, [r[0] for r in rng], [r[1] for r in rng], V, SHIFT))
    return out


def _as_mask(m):
    """A step's output as uint8 [B, V]: packed int32 words (unpack=False) expanded."""
    a = m.numpy()
    if a.dtype == np.int32:
        a = np.unpackbits(a.view(np.uint8), axis=1, bitorder="little")[:, :V]
    return a.copy()


def _worker(rank, world, port, halo, reduce, outdir, fused=False, grow=False, unpack=True):
    import torch.distributed as dist

    from fmidx.sharding import ShardedDecoder, shard_corpus

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    docs, patterns, steps = make_case()
    shard_docs_, _ = shard_corpus(docs, world, rank, halo)
    shard = (OracleShardFused if fused else OracleShard)(shard_docs_)
    dec = ShardedDecoder(shard, V, SHIFT, group=dist.group.WORLD, reduce=reduce, unpack=unpack)
    assert dec.fused == fused
    masks = [dec.start(patterns, "cpu").numpy().copy()]
    for tk in steps:
        masks.append(_as_mask(dec.step(torch.tensor(tk, dtype=torch.int64))))
    if grow:
        # the same decoder restarted with a batch three times larger: the payload and the
        # speculative gather size of the smaller batch must not be reused for it
        masks = [dec.start(patterns * 3, "cpu").numpy().copy()]
        for tk in steps:
            masks.append(dec.step(torch.tensor(tk * 3, dtype=torch.int64)).numpy().copy())
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.stack(masks))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, halo, reduce, fused=False, grow=False, unpack=True):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), halo, reduce, d, fused, grow, unpack), nprocs=world, join=True)
        return [np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)]


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("reduce", ["max_u8", "gather_bits", "sparse"])
def test_sharded_or_equals_unsharded(reduce, fused):
    """fused: one decode_step per step (the packed all_gather ships int32 words)."""
    docs, patterns, steps = make_case()
    want = np.stack(expected_masks(docs, patterns, steps))
    got = _run(2, 8 + 8 + 1, reduce, fused)      # halo >= longest pattern (7 + 8 steps) + 1
    for g in got:                          # every rank holds the reduced mask
        assert np.array_equal(g, want)


def test_sparse_exchange_packed_output():
    """unpack=False: the step returns the ORed rows as packed int32 words (what the
    processors' epilogue reads) -- equal, bit for bit, to the unsharded mask."""
    docs, patterns, steps = make_case()
    want = np.stack(expected_masks(docs, patterns, steps))
    for g in _run(2, 8 + 8 + 1, "sparse", fused=True, unpack=False):
        assert np.array_equal(g, want)


def test_sparse_exchange_survives_a_larger_batch():
    """a decoder whose batch grows (start() with more rows) must not
    reuse the smaller batch's payload buffer or speculative gather size."""
    docs, patterns, steps = make_case()
    want = np.stack(expected_masks(docs, patterns * 3, [tk * 3 for tk in steps]))
    for g in _run(2, 8 + 8 + 1, "sparse", fused=True, grow=True):
        assert np.array_equal(g, want)


def test_halo_is_required():
    docs, patterns, steps = make_case()
    want = np.stack(expected_masks(docs, patterns, steps))
    got = _run(2, 0, "max_u8")
    assert not np.array_equal(got[0], want)   # boundary-crossing n-grams are lost without a halo


def test_shard_docs_balanced():
    from fmidx.sharding import halo_tokens, shard_docs

    lens = [5, 1, 1, 9, 2, 2, 8, 3]
    parts = shard_docs(lens, 3)
    assert parts[0][0] == 0 and parts[-1][1] == len(lens)
    assert all(a <= b for a, b in parts) and all(parts[i][1] == parts[i + 1][0] for i in range(2))
    docs = [[1, 2], [3, 4, 5], [6]]
    assert halo_tokens(docs, 2, 4) == [3, 4, 5, 1]   # F continues with d1 then d0
    assert halo_tokens(docs, 0, 4) == []


def test_shard_text_device_is_shard_corpus_encoding():
    """shard_text_device slices T' on the device; the slice must be exactly
    index.py's encoding of shard_corpus's [halo] + docs[a:b] (+ sentinel)."""
    from fmidx.index import encode_corpus
    from fmidx.sharding import shard_corpus, shard_text_device

    docs, _, _ = make_case(11)
    data, beginnings, _ = encode_corpus(docs)
    text = torch.tensor(np.concatenate([data.astype(np.int64), [0]]), dtype=torch.int32)
    for world in (1, 2, 3, 5):
        for rank in range(world):
            for halo in (0, 1, 7, 40, 10 ** 6):
                sd, ab = shard_corpus(docs, world, rank, halo)
                want, _, _ = encode_corpus(sd)
                got, ab2 = shard_text_device(text, beginnings, world, rank, halo)
                assert ab == ab2
                assert got.tolist() == want.tolist() + [0], (world, rank, halo)


def test_halo_guard():
    """A row whose pattern outgrows halo - 1 tokens raises HaloExceeded before
    the step runs; restarts (token < 0) shorten rows and keep them legal."""
    from fmidx.sharding import HaloExceeded, ShardedDecoder

    docs, patterns, _ = make_case()
    shard = OracleShard(docs)
    pats = [p[:3] for p in patterns]
    dec = ShardedDecoder(shard, V, SHIFT, halo=6)
    dec.start(pats, "cpu")
    B = len(pats)
    tok = torch.full((B,), 5, dtype=torch.int64)
    dec.step(tok)                                   # 4 tokens
    dec.step(tok)                                   # 5 = halo - 1: still exact
    with pytest.raises(HaloExceeded):
        dec.step(tok)                               # 6 > halo - 1
    lo_before = dec.lo.clone()
    # the refused step left the state untouched; restarting every row makes it legal again
    assert torch.equal(dec.lo, lo_before)
    dec.step(torch.full((B,), -1, dtype=torch.int64))
    for _ in range(5):
        dec.step(tok)
    with pytest.raises(HaloExceeded):
        dec.step(tok)
    with pytest.raises(HaloExceeded):
        ShardedDecoder(shard, V, SHIFT, halo=3).start(pats + [[1, 2, 3]], "cpu")


def test_payload_facts_or():
    """The processors' per-row facts ride in the payload's facts area
    (pack_payload_host / fm_shard_pack_facts) and the OR pass ORs them over the
    parts: what fm_processor_shard_finish needs of the facts' sum (> 0)."""
    from fmidx.sharding import or_payloads_host, pack_payload_host, payload_facts_at, payload_header_words

    rng = np.random.default_rng(8)
    V, B, SH, P = 90, 13, 10, 3
    W = (V + 31) // 32
    bwt = rng.integers(0, V + SH, size=500)
    facts = [rng.integers(0, 2, size=(3, B)) * (rng.random((3, B)) < 0.3) for _ in range(P)]
    pays = []
    for p in range(P):
        lo = rng.integers(0, 450, size=B)
        hi = lo + rng.integers(0, 6, size=B)
        pays.append(pack_payload_host(lo, hi, bwt, np.zeros((B, W), dtype=np.int32), V, facts=facts[p]))
    m = max(q.numel() for q in pays)
    parts = torch.zeros((P, m), dtype=torch.int32)
    for p, q in enumerate(pays):
        parts[p, :q.numel()] = q
        assert int(q[payload_facts_at(B) + B + 4].item()) == int(facts[p][1, 4] != 0)
    assert payload_header_words(B) == payload_facts_at(B) + ((3 * B + 3) & ~3)
    fo = torch.empty((3, B), dtype=torch.int32)
    or_payloads_host(parts, B, V, SH, facts_out=fo)
    assert np.array_equal(fo.numpy(), (sum(f != 0 for f in facts) > 0).astype(np.int32))


def test_fixed_slot_payload_reads_like_compact():
    """fm_decode_step_payload's layout -- every row at a fixed slot H + b *
    round4(W), the unused words of a slot left as they were -- read by the
    host reader (and, on the GPU, fm_shard_or_rows / _peers, which follow the
    same desc / off words) gives what the compact payload of the same rows
    gives, for every row kind: empty, a slice narrower than W, a bitmap."""
    from fmidx.sharding import or_payloads_host, pack_payload_host

    rng = np.random.default_rng(4)
    V, B, SH = 200, 24, 10
    W = (V + 31) // 32
    n = 3000
    bwt = rng.integers(0, V + SH, size=n)
    lo = rng.integers(0, n - 40, size=B)
    width = rng.choice([0, 1, 3, W - 1, W, W + 9, 37], size=B)
    hi = lo + width
    bits = np.zeros((B, W * 32), dtype=np.uint8)
    for b in range(B):
        t = bwt[lo[b]:hi[b]] - SH
        bits[b, t[(t >= 0) & (t < V)]] = 1
    words = np.packbits(bits, axis=1, bitorder="little").view(np.int32)
    compact = pack_payload_host(lo, hi, bwt, words, V)
    from fmidx.sharding import payload_header_words

    H = payload_header_words(B)
    W4 = (W + 3) & ~3
    fixed = rng.integers(-2**31, 2**31, size=H + B * W4).astype(np.int64).astype(np.uint32)   # garbage
    c = compact.numpy().view(np.uint32)
    fixed[:4] = [H + B * W4, B, W, c[3]]
    for b in range(B):
        d, o = int(c[4 + b]), int(c[4 + B + b])
        cnt = d & 0x7FFFFFFF
        fixed[4 + b] = d
        fixed[4 + B + b] = H + b * W4
        fixed[H + b * W4:H + b * W4 + cnt] = c[o:o + cnt]
    got = or_payloads_host(torch.from_numpy(fixed.view(np.int32)).unsqueeze(0), B, V, SH)
    want = or_payloads_host(compact.unsqueeze(0), B, V, SH)
    assert torch.equal(got, want)
    assert torch.equal(want, torch.from_numpy(bits[:, :V]))


def test_decoder_default_exchange_without_rccl():
    """reduce="auto" (the default) is the peer exchange only over an RCCL group of more than one
    rank; a single process (group None) resolves to the plain max_u8 path."""
    from fmidx.sharding import ShardedDecoder

    class _Shard:   # only the attributes the constructor reads
        pass

    assert ShardedDecoder(_Shard(), 16, 0).reduce == "max_u8"
    with pytest.raises(ValueError):
        ShardedDecoder(_Shard(), 16, 0, reduce="ring")


def test_auto_exchange_needs_one_host(monkeypatch):
    """"auto" picks the peer exchange (hipIpc mappings) only when every
    rank of an RCCL group runs on ONE host; ranks on two nodes, or another
    backend, fall back to max_u8 (ShardedDecoder) / sparse (ShardedIndex)."""
    import torch.distributed as dist

    import fmidx.sharding as S

    class _Shard:
        device = 0

    hosts = {"ids": ["a/boot", "a/boot"]}
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "nccl")
    monkeypatch.setattr(dist, "get_world_size", lambda g=None: 2)

    def gather(out, obj, group=None):
        out[:] = hosts["ids"]

    monkeypatch.setattr(dist, "all_gather_object", gather)
    g = object()
    assert S.peer_capable(g)
    assert S.ShardedDecoder(_Shard(), 16, 0, group=g).reduce == "peer"
    assert S.ShardedIndex(_Shard(), [], group=g).exchange == "peer"
    hosts["ids"] = ["a/boot", "b/boot"]                     # two nodes
    assert not S.peer_capable(g)
    assert S.ShardedDecoder(_Shard(), 16, 0, group=g).reduce == "max_u8"
    assert S.ShardedIndex(_Shard(), [], group=g).exchange == "sparse"
    monkeypatch.setattr(dist, "get_backend", lambda g=None: "gloo")
    hosts["ids"] = ["a/boot", "a/boot"]
    assert not S.peer_capable(g)
    assert S.ShardedIndex(_Shard(), [], group=None).exchange == "sparse"
    assert isinstance(S.host_identity(), str)


def test_decoder_check_modes():
    """check="sync" (the default: a flag-barrier step raises at the step that timed
    out) or "deferred" (the opt-in of the previous behaviour); nothing else."""
    from fmidx.sharding import ShardedDecoder

    class _Shard:
        pass

    assert ShardedDecoder(_Shard(), 16, 0).check == "sync"
    assert ShardedDecoder(_Shard(), 16, 0, check="deferred").check == "deferred"
    with pytest.raises(ValueError):
        ShardedDecoder(_Shard(), 16, 0, check="never")
