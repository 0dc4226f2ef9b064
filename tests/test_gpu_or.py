"""fm_or_bits (csrc/shard.hip), the exchange step of doc-range sharding
(SURVEY §8e): the OR of P shards' bit-packed rows, as uint8 [B, V] 0/1 or as
packed words, against torch on random words -- both kernel shapes (16-B loads
when rows hold a multiple of 4 words, word loads otherwise), part counts
around the 8-load batch, vocab tails that end inside a 16-token chunk, row
strides wider than the vocab and a misaligned output."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    return torch.device("cuda:0")


def _expect(parts, V):
    import torch

    x = parts[0].clone()
    for p in parts[1:]:
        x |= p
    bits = ((x.to(torch.int64) & 0xFFFFFFFF).unsqueeze(-1) >> torch.arange(32, device=x.device)) & 1
    return x, bits.reshape(x.shape[0], -1)[:, :V].to(torch.uint8)


@pytest.mark.parametrize("P,B,V", [(1, 3, 17), (8, 5, 128256), (9, 4, 128256), (3, 7, 8192 * 2 + 33),
                                   (16, 2, 32 * 4 * 256), (5, 6, 100), (2, 1, 32 * 3 + 5), (11, 3, 151936)])
def test_or_bits_vs_torch(dev, P, B, V):
    import torch

    from fmidx.sharding import or_bits

    W = (V + 31) // 32
    g = torch.Generator(device="cpu").manual_seed(P * 1000 + V)
    # sparse words (most rows of a real step are nearly empty) and dense ones
    raw = torch.randint(-(1 << 31), 1 << 31, (P, B, W), generator=g, dtype=torch.int64)
    keep = torch.rand((P, B, W), generator=g) < 0.3
    parts = torch.where(keep, raw, torch.zeros_like(raw)).to(torch.int32).to(dev).contiguous()
    words, want = _expect(parts, V)
    assert torch.equal(or_bits(parts, V), want)
    assert torch.equal(or_bits(parts, V, unpack=False), words)
    # a row stride wider than the vocab, and an output that starts 1 byte into its allocation
    wide = torch.full((B, V + 48), 7, dtype=torch.uint8, device=dev)
    or_bits(parts, V, out=wide[:, :V])
    assert torch.equal(wide[:, :V], want) and bool((wide[:, V:] == 7).all())
    skew = torch.full((B, V + 17), 7, dtype=torch.uint8, device=dev)
    or_bits(parts, V, out=skew[:, 1:V + 1])
    assert torch.equal(skew[:, 1:V + 1], want) and bool((skew[:, 0] == 7).all())
    wide_w = torch.full((B, W + 4), 5, dtype=torch.int32, device=dev)
    or_bits(parts, V, out=wide_w[:, :W], unpack=False)
    assert torch.equal(wide_w[:, :W], words) and bool((wide_w[:, W:] == 5).all())


def test_or_bits_rejects_short_rows(dev):
    import torch

    from fmidx import FMIndexError
    from fmidx.sharding import or_bits

    parts = torch.zeros((2, 3, 4), dtype=torch.int32, device=dev)
    with pytest.raises(FMIndexError):
        or_bits(parts, 200)                      # 4 words cannot hold 200 tokens
    with pytest.raises(ValueError):
        or_bits(parts, 100, out=torch.empty((3, 100), dtype=torch.uint8, device=dev)[:, :50])
    np.testing.assert_array_equal(or_bits(parts, 100).cpu().numpy(), np.zeros((3, 100), np.uint8))


@pytest.mark.parametrize("V,B", [(100, 64), (128256, 64), (151936, 64), (128256, 320)])
@pytest.mark.parametrize("world", [2, 5])
def test_sparse_exchange_equals_dense_or_and_unsharded(dev, V, B, world):
    """fm_shard_pack + fm_shard_or_rows (the sparse C4 exchange) against the
    dense exchange (fm_or_bits over every shard's packed rows) and the
    unsharded index's mask, over doc-range shards with a halo: rows from
    empty to the full range, so both payload kinds (BWT slice, bitmap) occur;
    the gathered payloads are padded to the largest, as the all_gather does.
    B > 256 takes the OR pass's 256-thread workgroups (or_threads)."""
    import torch

    from fmidx.index import FMIndex
    from fmidx.sharding import or_bits, or_payloads, or_peer_payloads, payload_capacity, shard_corpus

    rng = np.random.default_rng(V + world)
    vocab_used = min(V, 3000)
    docs = [rng.integers(0, vocab_used, size=int(rng.integers(5, 400))).tolist() for _ in range(300)]
    # a repeated phrase so some patterns are wide on every shard
    for d in docs[::3]:
        d[:4] = [1, 2, 3, 4]
    F = [t for d in reversed(docs) for t in d]
    pats = [[]] + [[1, 2]] + [[1]] + [F[s:s + int(rng.integers(1, 5))] for s in rng.integers(0, len(F) - 8, B - 4)]
    pats.append([vocab_used + 7])                 # never in the corpus: empty everywhere
    full = FMIndex()
    full.initialize(docs, in_memory=True)
    lo, hi = full.get_range_batch(pats, 10)
    want = full.allowed_mask(torch.tensor(lo.astype(np.int64), device=dev), torch.tensor(hi.astype(np.int64), device=dev),
                             V, 10)
    W = (V + 31) // 32
    payloads, packed = [], []
    for r in range(world):
        sd, _ = shard_corpus(docs, world, r, 8)
        ix = FMIndex()
        ix.initialize(sd, in_memory=True)
        slo, shi = ix.get_range_batch(pats, 10)
        lo_t = torch.tensor(slo.astype(np.int64), device=dev)
        hi_t = torch.tensor(shi.astype(np.int64), device=dev)
        bits = ix.allowed_mask(lo_t, hi_t, V, 10, packed=True)
        packed.append(bits)
        pay = ix.shard_pack(lo_t, hi_t, bits, V)
        used = int(pay[0].item())
        assert used % 4 == 0 and used <= pay.numel()
        desc = pay[4:4 + B].cpu().numpy().view(np.uint32)
        widths = (np.minimum(shi, ix.size()) - slo).astype(np.int64)
        np.testing.assert_array_equal(desc >> 31, (widths >= W).astype(np.uint32))
        payloads.append(pay[:used])
        del ix
    m = max(p.numel() for p in payloads)
    parts = torch.zeros((world, m), dtype=torch.int32, device=dev)
    for r, p in enumerate(payloads):
        parts[r, :p.numel()] = p
    got = or_payloads(parts, B, V, 10)
    dense = or_bits(torch.stack(packed).contiguous(), V)
    assert torch.equal(dense, want)
    assert torch.equal(got, want)
    assert torch.equal(or_payloads(parts, B, V, 10, unpack=False), or_bits(torch.stack(packed).contiguous(), V,
                                                                           unpack=False))
    if V > 1000:   # most rows ship a slice, not a 16-KB bitmap
        assert sum(p.numel() for p in payloads) * 4 < world * B * W * 4 / 2
    # the peer exchange's pass: the same payloads read in place through a table of addresses
    cap = payload_capacity(B, V)
    bufs = [torch.zeros(cap, dtype=torch.int32, device=dev) for _ in range(world)]
    for bf, p in zip(bufs, payloads):
        bf[:p.numel()] = p
    ptrs = torch.tensor([bf.data_ptr() for bf in reversed(bufs)], dtype=torch.int64, device=dev)
    assert torch.equal(or_peer_payloads(ptrs, cap, B, V, 10), want)       # the OR does not care for order
    assert torch.equal(or_peer_payloads(ptrs, cap, B, V, 10, unpack=False),
                       or_payloads(parts, B, V, 10, unpack=False))


def test_sparse_or_reads_nothing_past_a_short_gather(dev):
    """A gather shorter than a payload (SparseExchange's speculative size,
    redone in full afterwards) must not make fm_shard_or_rows read past the
    part: rows whose data does not fit are read as empty -- the same rule as
    the host reader."""
    import torch

    from fmidx.index import FMIndex
    from fmidx.sharding import or_payloads, or_payloads_host

    rng = np.random.default_rng(3)
    docs = [rng.integers(0, 300, size=int(rng.integers(5, 200))).tolist() for _ in range(200)]
    ix = FMIndex()
    ix.initialize(docs, in_memory=True)
    V, B = 400, 48
    F = [t for d in reversed(docs) for t in d]
    pats = [[]] * 6 + [F[s:s + 1] for s in rng.integers(0, len(F) - 2, B - 6)]
    lo, hi = ix.get_range_batch(pats, 10)
    lo_t = torch.tensor(lo.astype(np.int64), device=dev)
    hi_t = torch.tensor(hi.astype(np.int64), device=dev)
    bits = ix.allowed_mask(lo_t, hi_t, V, 10, packed=True)
    pay = ix.shard_pack(lo_t, hi_t, bits, V)
    used = int(pay[0].item())
    from fmidx.sharding import payload_header_words

    H = payload_header_words(B)
    for m in (H, H + 8, (H + used) // 2 // 4 * 4, used):
        parts = pay[:m].unsqueeze(0).contiguous()
        got = or_payloads(parts, B, V, 10)
        want = or_payloads_host(parts.cpu(), B, V, 10)
        assert torch.equal(got.cpu(), want), m
    full = or_payloads(pay[:used].unsqueeze(0).contiguous(), B, V, 10)
    assert torch.equal(full, ix.allowed_mask(lo_t, hi_t, V, 10))


@pytest.mark.parametrize("V", [100, 128256])
def test_decode_payload_equals_packed_decode_and_unsharded(dev, V):
    """fm_decode_step_payload (the decode kernel writing the exchange payload
    itself, fixed row slots): per shard the same new states as
    fm_decode_step_batch, and the in-place OR of the shards' payloads
    (fm_shard_or_rows_peers) equal to the unsharded index's mask after the
    same step -- over rows that restart, go empty, stay narrow and stay wide,
    for two steps (the payload buffer rewritten)."""
    import torch

    from fmidx.index import FMIndex
    from fmidx.sharding import or_peer_payloads, payload_capacity, shard_corpus

    rng = np.random.default_rng(V + 17)
    vocab_used = min(V, 3000)
    docs = [rng.integers(0, vocab_used, size=int(rng.integers(5, 400))).tolist() for _ in range(300)]
    for d in docs[::3]:
        d[:4] = [1, 2, 3, 4]
    F = [t for d in reversed(docs) for t in d]
    world, B, halo = 3, 64, 16
    starts = rng.integers(0, len(F) - 12, B)
    pats = [[]] + [[1]] + [[1, 2]] + [F[s:s + int(rng.integers(1, 4))] for s in starts[3:]]
    full = FMIndex()
    full.initialize(docs, in_memory=True)
    shards = []
    for r in range(world):
        sd, _ = shard_corpus(docs, world, r, halo)
        ix = FMIndex()
        ix.initialize(sd, in_memory=True)
        shards.append(ix)

    def ranges(ix):
        lo, hi = ix.get_range_batch(pats, 10)
        return torch.tensor(lo.astype(np.int64), device=dev), torch.tensor(hi.astype(np.int64), device=dev)

    states = [ranges(ix) for ix in shards]
    flo, fhi = ranges(full)
    cap = payload_capacity(B, V)
    bufs = [torch.full((cap,), -7, dtype=torch.int32, device=dev) for _ in range(world)]
    ptrs = torch.tensor([b.data_ptr() for b in bufs], dtype=torch.int64, device=dev)
    W = (V + 31) // 32
    for step in range(2):
        nxt = [F[s + len(p)] if s + len(p) < len(F) else -1 for s, p in zip(starts, pats)]
        tok = [(-1 if i % 11 == 5 else (vocab_used + 3 if i % 13 == 7 else t)) for i, t in enumerate(nxt)]
        tok_t = torch.tensor(tok, dtype=torch.int64, device=dev)
        new_states = []
        for r, ix in enumerate(shards):
            lo, hi = states[r]
            lo2, hi2 = torch.empty_like(lo), torch.empty_like(hi)
            ix.decode_step_payload(tok_t, lo, hi, lo2, hi2, bufs[r], V, 10, reset_below=0)
            plo, phi = torch.empty_like(lo), torch.empty_like(hi)
            bits = torch.empty((B, W), dtype=torch.int32, device=dev)
            ix.decode_step(tok_t, lo, hi, bits, V, 10, reset_below=0, lo_out=plo, hi_out=phi, packed=True)
            assert torch.equal(lo2, plo) and torch.equal(hi2, phi), (step, r)
            desc = bufs[r][4:4 + B].cpu().numpy().view(np.uint32)
            w = (np.minimum(hi2.cpu().numpy(), ix.size()) - lo2.cpu().numpy()).clip(min=0)
            sparse = (desc >> 31) == 0          # a row ships its slice only when narrower than a bitmap
            assert np.all(w[sparse] < W) and np.array_equal(desc[sparse], w[sparse]), (step, r)
            assert np.all(desc[~sparse] == (W | 0x80000000)), (step, r)
            assert sparse[w < min(W, 64)].all(), (step, r)      # narrow streamed rows never write a bitmap
            new_states.append((lo2, hi2))
        states = new_states
        fm = torch.empty((B, V), dtype=torch.uint8, device=dev)
        flo2, fhi2 = torch.empty_like(flo), torch.empty_like(fhi)
        full.decode_step(tok_t, flo, fhi, fm, V, 10, reset_below=0, lo_out=flo2, hi_out=fhi2)
        flo, fhi = flo2, fhi2
        assert torch.equal(or_peer_payloads(ptrs, cap, B, V, 10), fm), step
        pats = [([] if t < 0 else p + [t]) for p, t in zip(pats, tok)]
