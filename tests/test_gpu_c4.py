"""C4 (enwiki doc-range sharded 8 ways) proven exact at full scale
on one GPU.

The 4.4e9-token corpus (n > 2^32) is indexed once unsharded (the replica) to
record B = 256 rows' ranges and packed masks over 8 decode steps of the
bench's trace; the replica is then freed and the 8 doc-range shards (each
``[halo] + docs[a:b]``, one slice of T' built on the device by
``shard_text_device``, halo = 128 tokens as §8d specifies) are built one after
another.  Every shard decodes every step from its own search of the initial
patterns with the fused kernel writing bit-packed rows -- exactly what each
rank of the 8-GPU run does -- and ``fm_or_bits`` ORs the 8 shards' rows.  The
OR must equal the replica's mask on every step, bit for bit; emptiness too
(a replica range is empty iff every shard's is).  Reference: docs are
concatenated without separators (index.py:47-53), so n-grams cross shard
borders and only the halo keeps the OR exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHIFT = 10
V = 128256
WORLD = 8
HALO = 128


@pytest.mark.timeout(1200)
def test_c4_eight_shards_or_equals_unsharded_at_enwiki_scale():
    import torch

    from fmidx.fm_index import FMIndex
    from fmidx.sharding import or_bits, shard_docs, shard_text_device
    from fmidx.synth import decode_trace, markov_corpus_gpu

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda:0")
    if torch.cuda.get_device_properties(0).total_memory < (200 << 30):
        pytest.skip("needs a 288 GB MI355X")
    torch.cuda.empty_cache()
    B, S = 256, 8
    Wd = (V + 31) // 32
    text, beg = markov_corpus_gpu(4_400_000_000, V, 41, dev)
    n = text.numel()
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text)
    bwt = fm.device_bwt()
    assert bwt.numel() > (1 << 32)
    tokens, init, lo_hist, hi_hist, pats0 = decode_trace(fm, text, bwt, B, V, S, 4242, dev)
    assert max(len(p) for p in pats0) + S <= HALO - 1
    want = torch.empty((S + 1, B, Wd), dtype=torch.int32, device=dev)
    fm.allowed_mask(init[0], init[1], V, SHIFT, out=want[0], packed=True)
    for s in range(S):
        fm.allowed_mask(lo_hist[s], hi_hist[s], V, SHIFT, out=want[s + 1], packed=True)
    want_u8 = fm.allowed_mask(lo_hist[S - 1], hi_hist[S - 1], V, SHIFT)
    live = torch.cat([(init[1] > init[0]).unsqueeze(0), hi_hist > lo_hist])      # [S + 1, B]
    widths = (hi_hist - lo_hist).cpu().numpy()
    assert (widths == 0).any() and ((widths > 0) & (widths <= 512)).any() and (widths > 4096).any()
    del bwt, fm
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    lens = [len(p) for p in pats0]
    offs = torch.tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), device=dev)
    toks = torch.tensor([t for p in pats0 for t in p], dtype=torch.int64, device=dev)
    parts = torch.empty((S + 1, WORLD, B, Wd), dtype=torch.int32, device=dev)
    any_live = torch.zeros((S + 1, B), dtype=torch.bool, device=dev)
    width_sum = torch.zeros((S + 1, B), dtype=torch.int64, device=dev)
    cuts = shard_docs(np.diff(beg.cpu().numpy()), WORLD)
    assert all(b > a for a, b in cuts) and cuts[0][0] == 0 and cuts[-1][1] == beg.numel() - 1
    shard_rows = []
    for r in range(WORLD):
        t_r, (a, b) = shard_text_device(text, beg, WORLD, r, HALO)
        assert (a, b) == cuts[r]
        ix = FMIndex(device=0)
        ix.initialize_from_text_device(t_r)
        shard_rows.append(t_r.numel())
        del t_r
        lo = torch.zeros(B, dtype=torch.int64, device=dev)
        hi = torch.zeros(B, dtype=torch.int64, device=dev)
        ix.backward_search_batch(toks, offs, SHIFT, lo, hi)
        lo[0], hi[0] = 0, ix.size()            # the trace's empty-pattern row
        lo[1], hi[1] = 0, 0                    # its eos row
        ix.allowed_mask(lo, hi, V, SHIFT, out=parts[0, r], packed=True)
        any_live[0] |= hi > lo
        width_sum[0] += hi - lo
        lo2, hi2 = torch.empty_like(lo), torch.empty_like(hi)
        for s in range(S):
            ix.decode_step(tokens[s], lo, hi, parts[s + 1, r], V, SHIFT, reset_below=0, lo_out=lo2, hi_out=hi2,
                           packed=True)
            lo, lo2 = lo2, lo
            hi, hi2 = hi2, hi
            any_live[s + 1] |= hi > lo
            width_sum[s + 1] += hi - lo
        torch.cuda.synchronize()
        del ix, lo, hi, lo2, hi2
        torch.cuda.empty_cache()
    # every token of T' is in exactly one shard's own region, plus 8 - 1 halos and 8 sentinels
    assert sum(shard_rows) == n + (WORLD - 1) * HALO + WORLD - 1
    for s in range(S + 1):
        got = or_bits(parts[s].contiguous(), V, unpack=False)
        bad = torch.nonzero((got != want[s]).any(1)).flatten()
        assert bad.numel() == 0, f"step {s}: OR of the shards differs from the replica on rows {bad[:8].tolist()}"
    assert torch.equal(or_bits(parts[S].contiguous(), V), want_u8)      # the uint8 [B, V] the processors read
    assert torch.equal(any_live, live)
    # counts: every occurrence of the replica is in some shard (halo duplicates add, never remove)
    rep_w = torch.cat([(init[1] - init[0]).unsqueeze(0), hi_hist - lo_hist])
    assert bool((width_sum >= rep_w).all())
