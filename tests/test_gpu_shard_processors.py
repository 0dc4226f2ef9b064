"""The logits processors over a doc-range sharded corpus (BASELINE
configs[3]) on ONE GPU: the 8 shards of a corpus (halo 64) are built side by
side, one processor per shard (fmidx.sharding.ShardedIndex, no process
group), and every call is driven as the 8 ranks would run it -- each shard's
fm_processor_shard_prep, the facts summed and the allowed bits ORed (the dense
exchange and the sparse one, which must agree), each shard's
fm_processor_shard_finish -- against the unsharded processor of the same class
(device path) and its host path, bit for bit, over generations with beam
reordering, eos / pad rows, think / system tokens, force_decoding_from and
always_allow_eos.  Every shard must return the same output."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

WORLD, HALO, V = 8, 64, 128256


def _corpus(seed):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(600):
        ln = int(rng.integers(20, 400))
        tok = int(rng.integers(0, 2000))
        d = []
        for _ in range(ln):
            d.append(tok)
            tok = (tok * 31 + 7) % 2000 if rng.random() < 0.6 else int(rng.integers(0, 2000))
        docs.append(d)
    for d in docs[::5]:                 # a phrase shared by many docs: wide ranges on every shard
        d[:5] = [3, 4, 5, 6, 7]
    return docs


@pytest.fixture(scope="module")
def indexes():
    from fmidx.index import FMIndex
    from fmidx.sharding import shard_corpus

    docs = _corpus(3)
    opts = {"cache_min": 8, "bm_log2": 6}   # cache / transitions / hierarchy exist on a small corpus
    full = FMIndex(options=opts)
    full.initialize(docs, in_memory=True)
    shards = []
    for r in range(WORLD):
        sd, _ = shard_corpus(docs, WORLD, r, HALO)
        ix = FMIndex(options=opts)
        ix.initialize(sd, in_memory=True)
        shards.append(ix)
    assert full.stats()["cache_nodes"] > 1
    return docs, full, shards


def _drive(procs, ids, scores):
    """One call of the sharded processors as WORLD ranks would run it."""
    from fmidx.sharding import or_bits, or_payloads

    cfgs = [p._prep_config(scores.dtype) for p in procs]
    hs = [p._dev.prep(ids, scores, c) for p, c in zip(procs, cfgs)]
    facts = torch.stack([h["facts"] for h in hs]).sum(0).to(torch.int32).contiguous()
    B, Vs = hs[0]["B"], hs[0]["V"]
    W = (Vs + 31) // 32
    dense = or_bits(torch.stack([h["bits"][:, :W] for h in hs]).contiguous(), Vs, unpack=False)
    # the payloads carry each shard's facts (fm_shard_pack_facts); the OR pass ORs them
    pays = [p._dev.index.shard_pack(h["mlo"], h["mhi"], h["bits"], Vs, facts=h["facts"]) for p, h in zip(procs, hs)]
    pays = [q[:int(q[0].item())] for q in pays]
    m = max(q.numel() for q in pays)
    parts = torch.zeros((len(pays), m), dtype=torch.int32, device=ids.device)
    for r, q in enumerate(pays):
        parts[r, :q.numel()] = q
    f_or = torch.empty((3, B), dtype=torch.int32, device=ids.device)
    sparse = or_payloads(parts, B, Vs, 10, unpack=False, facts_out=f_or)
    assert torch.equal(dense, sparse)
    assert torch.equal(f_or, (facts > 0).to(torch.int32))
    # even shards finish from the summed facts (the dense exchange's all_reduce), odd ones from the
    # payload's ORed facts (the sparse / peer exchanges): every output must be the same
    outs = [p._dev.finish(h, facts.clone() if r % 2 == 0 else f_or.clone(), sparse)
            for r, (p, h) in enumerate(zip(procs, hs))]
    for o in outs[1:]:
        assert torch.equal(o.view(torch.int16 if o.dtype != torch.float32 else torch.int32),
                           outs[0].view(torch.int16 if o.dtype != torch.float32 else torch.int32))
    return outs[0]


@pytest.mark.parametrize("variant", ["qwen", "causal", "seq"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sharded_processors_equal_unsharded(indexes, variant, dtype):
    import fmidx.processors as P
    from fmidx.sharding import ShardedIndex

    docs, full, shards = indexes
    occ = full.occurring_distinct
    rng = np.random.default_rng(101)
    F = [t for d in reversed(docs) for t in d]
    beams, groups = 4, 8
    B = beams * groups
    iv = torch.int32 if dtype == torch.float32 else torch.int16
    marker = [151645, 198, 151644, 77091, 198] if variant == "qwen" else [78191, 128007, 271]
    think = [151667, 271, 151668, 271]
    for cfg in range(2):
        kw = dict(num_beams=beams, pad_token_id=0, eos_token_id=2,
                  force_decoding_from=[F[11], F[12]] if cfg == 1 else None,
                  always_allow_eos=cfg == 1)
        if variant == "qwen":
            mk = lambda index: P.QwenIndexBasedLogitsProcessor(index=index, min_new_tokens=3,  # noqa: E731
                                                               length_reward_factor=1.5, **kw)
        elif variant == "causal":
            mk = lambda index: P.CausalIndexBasedLogitsProcessor(index=index, model_name="llama-3",  # noqa: E731
                                                                 length_reward_factor=1.5, **kw)
        else:
            mk = lambda index: P.SeqIndexBasedLogitsProcessor(index=index, **kw)  # noqa: E731
        ref_p, host_p = mk(full), mk(full)
        host_p._dev = None
        procs = [mk(ShardedIndex(s, occ, halo=HALO)) for s in shards]
        assert all(type(p._dev).__name__ == "_ShardedDeviceStep" for p in procs)
        starts = rng.integers(0, len(F) - 80, size=B)
        if variant == "seq":
            prompt, sents = [], [[1] for _ in range(B)]           # the decoder start token
        else:
            prompt = [int(x) for x in rng.integers(100, 200, size=4)] + marker
            sents = [[] for _ in range(B)]
            if variant == "qwen":
                for b in range(B):
                    sents[b] = [list(think), [5, 6, 151668, 271], [5, 6, 7, 8]][b % 3]
        for step in range(8):
            perm = np.concatenate([g * beams + rng.permutation(beams) for g in range(groups)])
            sents = [list(sents[i]) for i in perm]
            starts = starts[perm]
            for b in range(B):
                r = rng.random()
                if r < 0.78:
                    sents[b].append(F[(int(starts[b]) + len(sents[b])) % len(F)])
                elif r < 0.86:
                    sents[b].append(int(rng.integers(0, 2000)))
                elif r < 0.9:
                    sents[b].append(2)
                elif r < 0.93:
                    sents[b].append(0)
                else:
                    sents[b].append(int(rng.integers(5000, 6000)))      # never in the corpus
            ids = torch.tensor([prompt + s for s in sents], dtype=torch.int64).cuda()
            scores = torch.from_numpy(rng.standard_normal((B, V)).astype(np.float32)).to(dtype).cuda()
            want = ref_p(ids, scores.clone())
            host = host_p(ids, scores.clone())
            got = _drive(procs, ids, scores.clone())
            assert torch.equal(want.view(iv), host.view(iv)), (variant, cfg, step, "device vs host")
            assert torch.equal(got.view(iv), want.view(iv)), (variant, cfg, step)
        assert all(p._dev.prev_ids is not None for p in procs)     # the incremental state was kept


def test_sharded_processor_guards(indexes):
    """A pattern longer than the halo allows raises HaloExceeded; stop_at_count
    (a count, inflated by halo duplicates) is refused."""
    import fmidx.processors as P
    from fmidx import FMIndexError
    from fmidx.sharding import HaloExceeded, ShardedIndex

    docs, full, shards = indexes
    occ = full.occurring_distinct
    F = [t for d in reversed(docs) for t in d]
    ids = torch.tensor([[1] + F[100:100 + HALO + 2]], dtype=torch.int64).cuda()
    scores = torch.zeros((1, V), dtype=torch.float32).cuda()
    procs = [P.SeqIndexBasedLogitsProcessor(index=ShardedIndex(s, occ, halo=HALO), num_beams=1) for s in shards]
    with pytest.raises(HaloExceeded):
        _drive(procs, ids, scores)
    procs = [P.SeqIndexBasedLogitsProcessor(index=ShardedIndex(s, occ, halo=HALO), num_beams=1, stop_at_count=2)
             for s in shards]
    with pytest.raises(FMIndexError):
        _drive(procs, ids[:, :5], scores)


def test_sparse_exchange_over_rccl_world_one(indexes):
    """The RCCL code path of the sparse exchange (SparseExchange: the sizes
    all_gather, the speculative payload gather + OR, the re-issue when a
    payload outgrows the guess) and of ShardedIndex.or_bits, on a world of
    one rank: ShardedDecoder(reduce="sparse") over the whole corpus as its
    only shard == the unsharded masks, and the sharded processor == the
    unsharded one."""
    import socket

    import torch.distributed as dist

    import fmidx.processors as P
    from fmidx.sharding import ShardedDecoder, ShardedIndex

    docs, full, shards = indexes
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    try:
        rng = np.random.default_rng(7)
        F = [t for d in reversed(docs) for t in d]
        B = 64
        starts = rng.integers(0, len(F) - 40, size=B)
        pats = [F[a:a + 3] for a in starts]
        dec = ShardedDecoder(full, V, 10, group=dist.group.WORLD, reduce="sparse", halo=None)
        dec.start(pats, "cuda")
        for step in range(12):
            tok = [F[a + 3 + step] if rng.random() < 0.8 else int(rng.integers(0, 2000)) for a in starts]
            if step == 6:          # every row restarts: wide ranges, a payload far above the guess
                tok = [-1] * B
            got = dec.step(torch.tensor(tok, dtype=torch.int64, device="cuda"))
            want = full.allowed_mask(dec.lo, dec.hi, V, 10)
            assert torch.equal(got, want), step
        assert dec._xchg.respecified >= 1          # the restart step outgrew the speculative size
        # the peer exchange with its stream-ordered RCCL barrier and with the flag barrier (a world of
        # one: the own buffer and flag word only)
        for pb, graph in (("collective", False), ("flags", False), ("flags", True)):
            pdec = ShardedDecoder(full, V, 10, group=dist.group.WORLD, reduce="peer", halo=None, peer_barrier=pb,
                                  graph=graph)
            pdec.start(pats, "cuda")
            for step in range(6):
                tok = [F[a + 3 + step] if rng.random() < 0.8 else -1 for a in starts]
                got = pdec.step(torch.tensor(tok, dtype=torch.int64, device="cuda"))
                assert torch.equal(got, full.allowed_mask(pdec.lo, pdec.hi, V, 10)), (pb, graph, step)
            assert pdec._peer.errors() == 0
            assert (pdec._g is not None) == graph
            # a larger batch on the same decoder: the exchange is rebuilt with room for it
            pats2 = [F[a:a + 2] for a in rng.integers(0, len(F) - 40, size=3 * B)]
            pdec.start(pats2, "cuda")
            got = pdec.step(torch.tensor([F[0]] * (3 * B), dtype=torch.int64, device="cuda"))
            assert pdec._peer.rows >= 3 * B
            assert torch.equal(got, full.allowed_mask(pdec.lo, pdec.hi, V, 10)), pb
            pdec.close()
            assert pdec._peer is None
        occ = full.occurring_distinct
        mk = lambda index: P.SeqIndexBasedLogitsProcessor(index=index, num_beams=1)  # noqa: E731
        ref = mk(full)
        calls = {"n": 0}
        real = {k: getattr(dist, k) for k in ("all_reduce", "all_gather", "all_gather_into_tensor", "barrier",
                                                "all_gather_object", "broadcast")}

        def counting(k):
            def f(*a, **kw):
                calls["n"] += 1
                return real[k](*a, **kw)
            return f

        for exchange, pb in (("sparse", "flags"), ("peer", "collective"), ("peer", "flags"), ("dense", "flags")):
            sidx = ShardedIndex(full, occ, group=dist.group.WORLD, exchange=exchange, peer_barrier=pb)
            sp = mk(sidx)
            for step in range(4):
                ids = torch.tensor([[1] + F[a:a + 2 + step] for a in starts[:8]], dtype=torch.int64).cuda()
                scores = torch.from_numpy(rng.standard_normal((8, V)).astype(np.float32)).cuda()
                want_out = ref(ids, scores.clone())
                # (the peer exchange maps its buffers at the first call: count from the second)
                for k in real:
                    setattr(dist, k, counting(k))
                calls["n"] = 0
                try:
                    got_out = sp(ids, scores.clone())
                finally:
                    for k, f in real.items():
                        setattr(dist, k, f)
                assert torch.equal(got_out.view(torch.int32), want_out.view(torch.int32)), (exchange, pb, step)
                if step and exchange == "peer" and pb == "flags":
                    # the facts ride in the payload, the flag barrier replaces the collective: none at all
                    assert calls["n"] == 0, (exchange, pb, calls["n"])
                if step and exchange == "peer" and pb == "collective":
                    assert calls["n"] == 1, (exchange, pb, calls["n"])   # the barrier alone: facts in the payload
            # the sparse exchange with a larger batch on the same index (its payload and speculative
            # gather size are rebuilt for it: ADVICE r4)
            ids = torch.tensor([[1] + F[a:a + 3] for a in rng.integers(0, len(F) - 40, size=40)],
                               dtype=torch.int64).cuda()
            scores = torch.from_numpy(rng.standard_normal((40, V)).astype(np.float32)).cuda()
            assert torch.equal(sp(ids, scores.clone()).view(torch.int32), ref(ids, scores.clone()).view(torch.int32))
            # the host path over the shard: a row without the end marker, boosts past the float range
            _qwen_host_path(full, sidx, F, rng)
            sidx.close()
    finally:
        dist.destroy_process_group()


def _qwen_host_path(full, sidx, F, rng):
    """Qwen inputs the device path hands to the host path (a row without the
    end marker; 10 * 2^k past fp32's range: the reference's RuntimeError),
    and a bf16 call whose boosts are inf (written on the device, as the
    reference writes them): the processor over ShardedIndex gives the
    unsharded processor's outcome, bit for bit or the same exception."""
    import fmidx.processors as P

    marker, think = [151645, 198, 151644, 77091, 198], [151667, 271, 151668, 271]
    kw = dict(num_beams=1, min_new_tokens=3, always_allow_eos=True, length_reward_factor=2.0)
    ref_p = P.QwenIndexBasedLogitsProcessor(index=full, **kw)
    sh_p = P.QwenIndexBasedLogitsProcessor(index=sidx, **kw)
    B = 6
    st = rng.integers(0, len(F) - 200, size=B)
    eos_rows = [b for b in range(B) if b % 3 == 1]

    def rows(k, drop_marker=False):
        out = []
        for b in range(B):
            s = [int(x) for x in F[int(st[b]):int(st[b]) + 5]]
            if b in eos_rows:
                s = [int(x) for x in rng.integers(0, 2000, size=k - 1)] + [2]
            out.append([100, 101] + marker + think + s)
        w = max(len(r) for r in out)
        out = [r + [0] * (w - len(r)) for r in out]
        if drop_marker:
            out[2][2:7] = [9, 9, 9, 9, 9]
        return out

    def outcome(p, ids, sc):
        try:
            o = p(ids, sc.clone())
        except Exception as e:  # noqa: BLE001 -- the reference's exception is the expected outcome
            return type(e).__name__, str(e)
        return "ok", o.view(torch.int32 if o.dtype == torch.float32 else torch.int16).cpu()

    for name, ids_l, dt in (("k>=125 bf16", rows(130), torch.bfloat16), ("k>=125 fp32", rows(130), torch.float32),
                            ("no marker", rows(6, True), torch.bfloat16), ("ordinary", rows(6), torch.float32)):
        ids = torch.tensor(ids_l, dtype=torch.int64).cuda()
        sc = torch.from_numpy(rng.standard_normal((B, V)).astype(np.float32)).to(dt).cuda()
        want, got = outcome(ref_p, ids, sc), outcome(sh_p, ids, sc)
        assert want[0] == got[0], (name, want[0], got[0], got[1] if got[0] != "ok" else "")
        if want[0] == "ok":
            assert torch.equal(want[1], got[1]), name
        else:
            assert want[1] == got[1], name
        if name == "k>=125 fp32":
            assert want[0] == "RuntimeError", want
        if name == "k>=125 bf16":
            assert want[0] == "ok" and torch.isinf(ref_p(ids, sc.clone()).float()).any()
