"""Doc-range sharding of the FM-index across GPUs.

Every rank holds the FM-index of a contiguous range of documents plus a
*halo*; every rank runs all B rows against its shard; the per-shard
allowed-token masks are OR-reduced across ranks.

Exactness.  Patterns match in F = reverse(T') = d_m ... d_1 d_0 (index.py
reverses every doc and concatenates them without separators, index.py:47-53),
so an n-gram may run across document boundaries.  Shard r owning docs
[a, b) is built over the pseudo-corpus ``[halo] + docs[a:b]`` where ``halo``
is the first H tokens that follow its region in F, i.e. d_{a-1} d_{a-2} ...
Its own F_r = d_{b-1} ... d_a ++ halo is a contiguous substring of F, so every
occurrence it finds (and the token that follows it) is a real occurrence in F;
and every occurrence in F that *starts* inside shard r's region lies, with
its next token, inside F_r when H >= Lmax + 1 (Lmax = longest pattern).
Hence OR over shards == the unsharded mask, bit for bit.  Ranges (low, high)
are shard-local SA coordinates and counts include halo duplicates, so only
masks / emptiness are comparable across shard layouts (the reference's only
count consumer, stop_at_count, is 0 at every call site).

The collective is the only data-path exchange: ``all_reduce(MAX)`` of the
uint8 [B, V] mask (0/1, so MAX == OR), ``all_gather`` of bit-packed masks
followed by a local OR (8x fewer bytes on the wire), or -- the default on the
GPU -- the sparse exchange: each rank ships, per row, its shard's BWT slice
when that is smaller than the row's bitmap, else the bitmap (fm_shard_pack;
most rows are a few rows wide on a shard), one tiny all_gather of the payload
sizes, one all_gather of the payloads (the largest rank's prefix), then one
fused OR / scatter / unpack pass (fm_shard_or_rows).  The peer exchange
(PeerExchange) ships nothing: every rank maps the others' payload buffers once
(hipIpc over xGMI) and, after one stream-ordered barrier, the OR pass reads
them in place (fm_shard_or_rows_peers) -- no host read of sizes, no gather.
"""
from __future__ import annotations

import bisect
import ctypes
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np


def shard_docs(lengths: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous doc ranges balanced by token count (boundaries at the
    k * total / world quantiles of the cumulative length)."""
    cum = np.concatenate([[0], np.cumsum(np.asarray(lengths, dtype=np.int64))])
    total = int(cum[-1])
    n = len(lengths)
    cuts = [0]
    for k in range(1, world):
        target = total * k / world
        i = int(np.searchsorted(cum, target, side="left"))
        i = min(max(i, cuts[-1]), n)
        cuts.append(i)
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def halo_tokens(docs: Sequence[Sequence[int]], a: int, H: int) -> List[int]:
    """The first H tokens that follow docs[a:] 's region in F: d_{a-1} d_{a-2} ..."""
    out: List[int] = []
    j = a - 1
    while j >= 0 and len(out) < H:
        out.extend(list(docs[j])[: H - len(out)])
        j -= 1
    return out


def shard_corpus(docs: Sequence[Sequence[int]], world: int, rank: int, halo: int):
    """The pseudo-corpus shard ``rank`` indexes: [halo] + docs[a:b]."""
    (a, b) = shard_docs([len(d) for d in docs], world)[rank]
    h = halo_tokens(docs, a, halo)
    return ([h] if h else []) + [list(d) for d in docs[a:b]], (a, b)


def shard_text_device(text, beginnings, world: int, rank: int, halo: int):
    """Shard ``rank``'s indexed text built on the device from the whole T'.

    ``text`` is T' (int32, sentinel last, index.py:47-53 encoding) and
    ``beginnings`` the doc offsets (index.py:50).  The encoding of
    ``[halo] + docs[a:b]`` (shard_corpus) is ONE slice of T': T' holds
    rev(d_0) rev(d_1) ..., and the halo -- the first H tokens of
    d_{a-1} d_{a-2} ... -- reversed is exactly the H tokens of T' before
    beginnings[a].  So T'_r = T'[max(0, beg[a] - H) : beg[b]] + sentinel, with
    no host copy of the corpus.  Returns (T'_r int32 on text.device, (a, b))."""
    import torch

    beg = np.asarray(beginnings.cpu() if hasattr(beginnings, "cpu") else beginnings, dtype=np.int64)
    a, b = shard_docs(np.diff(beg), world)[rank]
    lo = max(0, int(beg[a]) - int(halo))
    hi = int(beg[b])
    out = torch.empty(hi - lo + 1, dtype=torch.int32, device=text.device)
    out[:-1].copy_(text[lo:hi])
    out[-1] = 0
    return out, (a, b)


def host_identity() -> str:
    """This machine's identity: hostname + kernel boot id (two containers of one
    node share the boot id; two nodes never do)."""
    import socket

    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return f"{socket.gethostname()}/{boot}"


def peer_capable(group) -> bool:
    """True when the peer exchange can serve ``group``: an RCCL ("nccl") group of
    more than one rank whose ranks all run on ONE host -- the payload buffers are
    mapped through hipIpc handles, which do not cross nodes.  Collective (every
    rank of ``group`` calls it): the ranks' host identities are all_gathered."""
    if group is None:
        return False
    import torch.distributed as dist

    if dist.get_backend(group) != "nccl" or dist.get_world_size(group) <= 1:
        return False
    every = [None] * dist.get_world_size(group)
    dist.all_gather_object(every, host_identity(), group=group)
    return len(set(every)) == 1


class HaloExceeded(ValueError):
    """A row's pattern outgrew the shards' halo: OR over shards would no longer
    equal the unsharded mask (occurrences crossing a shard boundary by more
    than the halo are in no shard)."""


class ShardedDecoder:
    """Incremental constrained decoding over a doc-range shard.

    ``index`` is this rank's shard index with the batched API of
    :class:`fmidx.fm_index.FMIndex` (``get_range_batch``, ``decode_step`` or
    ``lf_step_batch`` + ``allowed_mask``); ``group`` a torch.distributed
    process group (None = single process, no collective).  State (lo, hi) per
    row is shard-local.

    With the fused ``decode_step`` a step is ONE launch (LF step + mask)
    writing into a persistent mask buffer -- bit-packed int32 [B, ceil(V/32)]
    when ``reduce="gather_bits"``, so the all_gather ships the kernel's own
    output -- and the (lo, hi) state ping-pongs between two buffers.  The mask
    ``step`` returns is that buffer (or, for gather_bits, a fresh tensor): it
    is valid until the next step.
    """

    def __init__(self, index, vocab: int, shift: int = 10, group=None, reduce: str = "auto",
                 halo: Optional[int] = None, peer_barrier: str = "flags", graph: bool = False,
                 spins: Optional[int] = None, check: str = "sync", unpack: bool = True):
        """reduce: "auto" (the default: "peer" with the flag barrier -- the fastest exact exchange,
        bench.py's sharded leg -- over an RCCL group of more than one rank whose ranks all run on
        one host (the IPC mappings do not cross nodes; same_host()); "max_u8" otherwise), "max_u8"
        (all_reduce MAX of the uint8 mask), "gather_bits"
        (all_gather of the packed rows + fm_or_bits), "sparse" (BWT slices /
        bitmaps per row, fm_shard_pack + all_gather + fm_shard_or_rows) or
        "peer" (the same payloads read in place over xGMI: PeerExchange, whose
        ``barrier`` is ``peer_barrier``, with at most ``spins`` flag polls).
        ``graph`` (peer + flags): the step -- the payload decode, the signal,
        the OR pass -- is captured into ONE HIP graph at its first call and
        replayed for every later step (the tokens copied into its static
        input); the step number and the buffer parity live on the device.
        ``check`` (flag barrier only): "sync" (the default) -- every step waits
        for its own OR pass (an event after it) and reads the exchange's error
        word before returning, so a step whose barrier timed out raises
        PeerBarrierTimeout and returns NO mask: masks are exact or absent;
        "deferred" -- no wait: the error word is read at the next call (and at
        close()), so the step that timed out has already handed back a mask
        that may be inexact (one stale mask at most) -- for callers that
        overlap the next step's host work with this step's GPU work and accept
        that contract.
        ``unpack`` (the "peer" and "sparse" exchanges): False makes ``step``
        return the ORed rows as packed int32 words [B, ceil(V/32)] (bit t of a
        row = token t) instead of the uint8 [B, V] mask -- what the processors'
        epilogue consumes -- so the OR pass writes V/8 bytes per row, not V."""
        self.index = index
        self.vocab = vocab
        self.shift = shift
        self.group = group
        if reduce == "auto":
            reduce = "peer" if peer_capable(group) else "max_u8"
        if reduce not in ("max_u8", "gather_bits", "sparse", "peer"):
            raise ValueError(reduce)
        if check not in ("sync", "deferred"):
            raise ValueError(check)
        if not unpack and reduce not in ("peer", "sparse"):
            raise ValueError("unpack=False: the peer and sparse exchanges only")
        self.unpack = unpack
        self.check = check
        self._ev = None        # the event a checked flag-barrier step waits on
        if graph and not (reduce == "peer" and peer_barrier == "flags"):
            raise ValueError("graph: only the peer exchange with the flag barrier holds no collective")
        self.reduce = reduce
        self.peer_barrier = peer_barrier
        self.graph = graph
        self.spins = spins
        self._g = None         # the captured step (graph=True) and its static token input
        self._g_tok = None
        self._peer = None      # its PeerExchange (reduce="peer")
        self.halo = halo
        self.fused = hasattr(index, "decode_step")
        self.lo = None
        self.hi = None
        self._buf = None
        self._plen = None      # per-row pattern length (device)
        self._bound = 0        # host upper bound of max(_plen)
        self._parts = None     # gathered packed rows of every rank (device path)
        self._out = None
        self._payload = None   # this rank's sparse-exchange payload
        self._xchg = None      # its SparseExchange
        self.exchange_words = []   # sparse: words every rank shipped, per step (host ints)

    def _check_halo(self):
        """Exactness needs every pattern to be at most halo - 1 tokens.  The
        host bound grows by one per step; only when it crosses the limit is
        the exact per-row maximum read back (one sync) -- restarts may have
        shortened the rows."""
        if self.halo is None or self._bound <= self.halo - 1:
            return
        exact = int(self._plen.max().item()) if self._plen.numel() else 0
        if exact > self.halo - 1:
            raise HaloExceeded(f"pattern of {exact} tokens needs a halo of >= {exact + 1} (shards built with "
                               f"{self.halo}); rebuild the shards with a larger halo or restart the row")
        self._bound = exact

    def start(self, patterns: Sequence[Sequence[int]], device):
        import torch

        lens = [len(p) for p in patterns]
        self._plen = torch.tensor(lens, dtype=torch.int64, device=device)
        self._bound = max(lens, default=0)
        self._check_halo()
        lo, hi = self.index.get_range_batch(patterns, self.shift)
        self.lo = torch.tensor(lo.astype(np.int64), device=device)
        self.hi = torch.tensor(hi.astype(np.int64), device=device)
        self._buf = None
        self._g = None         # the captured step names the old state buffers
        return self.mask()

    def step(self, tokens):
        """Append one token per row (token < 0: restart with an empty pattern).
        Raises HaloExceeded (before any work) when a row's pattern would be
        longer than the shards' halo allows."""
        import torch

        if self._plen is not None:
            plen = torch.where(tokens < 0, torch.zeros_like(self._plen), self._plen + 1)
            prev = (self._plen, self._bound)
            self._plen, self._bound = plen, self._bound + 1
            try:
                self._check_halo()
            except HaloExceeded:
                self._plen, self._bound = prev
                raise
        if not self.fused:
            self.index.lf_step_batch(tokens, self.lo, self.hi, self.shift, reset_below=0)
            return self.mask()
        if self.group is not None and self.reduce == "peer" and hasattr(self.index, "decode_step_payload"):
            return self._step_peer(tokens)
        packed = self.group is not None and self.reduce in ("gather_bits", "sparse", "peer")
        if self._buf is None:
            B = self.lo.numel()
            if packed:
                self._buf = torch.empty((B, (self.vocab + 31) // 32), dtype=torch.int32, device=self.lo.device)
            else:
                self._buf = torch.empty((B, self.vocab), dtype=torch.uint8, device=self.lo.device)
            self._lo2 = torch.empty_like(self.lo)
            self._hi2 = torch.empty_like(self.hi)
        self.index.decode_step(tokens, self.lo, self.hi, self._buf, self.vocab, self.shift, reset_below=0,
                               packed=packed, lo_out=self._lo2, hi_out=self._hi2)
        self.lo, self._lo2 = self._lo2, self.lo
        self.hi, self._hi2 = self._hi2, self.hi
        if self.group is not None and self.reduce == "sparse":
            return self._combine_sparse(self._buf)
        if self.group is not None and self.reduce == "peer":
            return self._combine_peer(self._buf)
        return self._combine(self._buf, packed)

    def _step_peer(self, tokens):
        """The peer exchange's step: the decode kernel writes this rank's payload
        itself (fixed row slots, fm_decode_step_payload: no pack pass), then the
        barrier and the in-place OR of every rank's payload.  With the flag
        barrier the state is updated in place and the payload buffer picked by
        the device counter, so the same launches serve every step (graph)."""
        import torch

        B = self.lo.numel()
        if self._peer is None or self._peer.rows < B:
            self.close()
            self._peer = PeerExchange(self.group, B, self.vocab, self.lo.device, barrier=self.peer_barrier,
                                      spins=self.spins)
            self._g = None
        self._peer.check()                 # a timed-out step before this one (check="deferred"): raise
        if self._out_stale(B, self.lo.device):
            self._out = self._new_out(B, self.lo.device)
            self._g = None
        if self.peer_barrier == "flags":
            px = self._peer

            def launch(tok, sync=False):
                px.flags_step(self.index, tok, self.lo, self.hi, self.vocab, self.shift, self._out,
                              unpack=self.unpack, sync=sync)

            if not self.graph:
                # one C call; with check="sync" it also waits for the step and reads the error word
                launch(tokens, sync=self.check == "sync")
                px.step += 1
                if self.check == "sync":
                    px.check()
                return self._out
            else:
                if self._g is None:
                    self._g_tok = torch.empty_like(tokens)
                    torch.cuda.synchronize(self.lo.device)
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g):
                        launch(self._g_tok)
                    self._g = g
                self._g_tok.copy_(tokens)
                self._g.replay()
            px.step += 1
            return self._checked(self._out)
        if self._buf is None:              # start() resets it: fresh second state buffers
            self._lo2 = torch.empty_like(self.lo)
            self._hi2 = torch.empty_like(self.hi)
            self._buf = ()
        pay = self._peer.payload()
        self.index.decode_step_payload(tokens, self.lo, self.hi, self._lo2, self._hi2, pay, self.vocab, self.shift,
                                       reset_below=0)
        self.lo, self._lo2 = self._lo2, self.lo
        self.hi, self._hi2 = self._hi2, self.hi
        return self._checked(self._peer(pay, B, self.vocab, self.shift, out=self._out, unpack=self.unpack))

    def _out_shape(self, B: int):
        return (B, self.vocab) if self.unpack else (B, (self.vocab + 31) // 32)

    def _out_stale(self, B: int, device) -> bool:
        return self._out is None or tuple(self._out.shape) != self._out_shape(B) or self._out.device != device

    def _new_out(self, B: int, device):
        import torch

        return torch.empty(self._out_shape(B), dtype=torch.uint8 if self.unpack else torch.int32, device=device)

    def _combine_peer(self, bits):
        import torch

        B = self.lo.numel()
        if self._peer is None or self._peer.rows < B:
            self.close()
            self._peer = PeerExchange(self.group, B, self.vocab, self.lo.device, barrier=self.peer_barrier,
                                      spins=self.spins)
        self._peer.check()
        pay = self._peer.payload()
        self.index.shard_pack(self.lo, self.hi, bits, self.vocab, payload=pay)
        if self._out_stale(B, pay.device):
            self._out = self._new_out(B, pay.device)
        return self._checked(self._peer(pay, B, self.vocab, self.shift, out=self._out, unpack=self.unpack))

    def _checked(self, out):
        """Exact or absent: with the flag barrier and check="sync", wait for the
        step's OR pass (an event recorded after it on the current stream) and
        read the error word -- a step whose barrier timed out raises
        PeerBarrierTimeout here and its mask is never returned."""
        if self.peer_barrier != "flags" or self.check != "sync" or self._peer is None:
            return out
        import torch

        if self._ev is None:
            self._ev = torch.cuda.Event()
        self._ev.record()
        self._ev.synchronize()
        self._peer.check()
        return out

    def close(self):
        """Release the peer exchange's mappings (collective: every rank calls it);
        raises PeerBarrierTimeout if one of its steps timed out."""
        self._g = None
        if self._peer is not None:
            px, self._peer = self._peer, None
            px.close()

    def _combine_sparse(self, bits):
        """The sparse exchange of this step's rows (new state self.lo/hi,
        their packed bits from the decode step)."""
        import torch

        self._payload = self.index.shard_pack(self.lo, self.hi, bits, self.vocab, payload=self._payload)
        B = self.lo.numel()
        if self._payload.is_cuda and self._out_stale(B, self._payload.device):
            self._out = self._new_out(B, self._payload.device)
        if self._xchg is None:
            self._xchg = SparseExchange(self.group)
            self.exchange_words = self._xchg.words
        return self._xchg(self._payload, B, self.vocab, self.shift, out=self._out if self._payload.is_cuda else None,
                          unpack=self.unpack)

    def local_mask(self):
        return self.index.allowed_mask(self.lo, self.hi, self.vocab, self.shift)

    def mask(self):
        return self._combine(self.local_mask(), False)

    def _combine(self, m, packed: bool):
        """OR of the ranks' masks: in place for max_u8; all_gather of the
        bit-packed rows (int32 words, or uint8 [B, V] packed here) otherwise."""
        if self.group is None:
            return m
        import torch
        import torch.distributed as dist

        if self.reduce == "max_u8":
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
            return m
        world = dist.get_world_size(self.group)
        if m.is_cuda and packed:
            # device path: one all_gather of the kernel's own int32 rows into a
            # [world, B, W] buffer, then ONE fused OR + unpack pass (fm_or_bits)
            B, W = m.shape
            if self._parts is None or self._parts.shape != (world, B, W):
                self._parts = torch.empty((world, B, W), dtype=torch.int32, device=m.device)
                self._out = torch.empty((B, self.vocab), dtype=torch.uint8, device=m.device)
            dist.all_gather_into_tensor(self._parts, m, group=self.group)
            or_bits(self._parts, self.vocab, out=self._out)
            return self._out
        # host tensors (gloo, CPU tests): the same exchange with torch ops.
        # int32 words in little-endian bit order are, byte for byte, pack_bits' layout.
        pk = m if packed else pack_bits(m)
        parts = [torch.empty_like(pk) for _ in range(world)]
        dist.all_gather(parts, pk, group=self.group)
        acc = parts[0].clone()
        for p in parts[1:]:
            acc |= p
        if packed:
            acc = acc.view(torch.uint8)
        return unpack_bits(acc, self.vocab)


class ShardedIndex:
    """This rank's doc-range shard as the ``index`` of the logits processors
    (fmidx.processors), so the reference's processors run over a corpus
    sharded across GPUs: each call runs the row bookkeeping and
    the pattern search on the shard, sums the shards' facts (count([last]) >
    0, range and distinct set non-empty) and ORs their allowed bits over
    ``group`` (RCCL), then decides and applies the boosts -- the same output
    on every rank, bit for bit the unsharded processor's.

    ``shard``: this rank's engine FMIndex (built from ``shard_text_device`` /
    ``shard_corpus`` with ``halo``).  ``occurring_distinct``: the WHOLE
    corpus's all-unigram list (index.py:67 -- it excludes BWT row n - 1 of
    the unsharded index, so it is not the union of the shards' lists; take it
    from the corpus's index metadata).  ``exchange``: "sparse" (per row the
    shard's BWT slice or bitmap, all_gathered), "peer" (the same payloads read
    in place over xGMI, PeerExchange; the facts all_reduce, issued after the
    pack, is its barrier) or "dense" (every row's bitmap).  A pattern
    longer than ``halo`` - 1 tokens raises HaloExceeded and stop_at_count must
    be 0 (counts include halo duplicates).  Inputs the device path hands to the
    processors' host path (rows without exactly one end marker, boosts outside
    the float range) run it over the shards: the host path's index calls
    become this class's sharded forms -- ``get_range_batch`` /
    ``allowed_mask`` on the shard, ``sum_counts`` (count([last]) summed over
    the ranks: zero exactly when the unsharded count is zero) and the allowed
    bits ORed over the ranks -- so such a call returns the unsharded host
    path's output, or raises where the reference raises.  Every rank makes the
    same calls in the same order (they depend on the inputs, not the shard).
    The default exchange ("auto") is the fastest exact one where it can run:
    "peer" with the flag barrier (no collective per exchange; a timed-out
    barrier raises PeerBarrierTimeout) over an RCCL group whose ranks share one
    host (peer_capable), "sparse" otherwise (another backend, or ranks on
    several nodes, where hipIpc mappings cannot reach).  The ``index.py`` query surface (get_range, distinct,
    ...) is the unsharded index's business and is not offered here."""

    sharded = True

    def __init__(self, shard, occurring_distinct, group=None, halo: Optional[int] = None, exchange: str = "auto",
                 shift: int = 10, peer_barrier: str = "flags", spins: Optional[int] = None):
        if exchange == "auto":
            exchange = "peer" if peer_capable(group) else "sparse"
        if exchange not in ("sparse", "dense", "peer"):
            raise ValueError(exchange)
        self.peer_barrier = peer_barrier
        self.spins = spins
        self._peer = None
        self._staged = False
        self.shard = shard
        self.occurring_distinct = list(occurring_distinct)
        self.group = group
        self.halo = halo
        self.exchange = exchange
        self.shift = shift
        self._payload = None
        self._parts = None
        self._xchg = None

    @property
    def device(self) -> int:
        return self.shard.device

    def sum_facts(self, facts):
        """SUM of every rank's int32 facts (in place)."""
        if self.group is not None:
            import torch.distributed as dist

            dist.all_reduce(facts, op=dist.ReduceOp.SUM, group=self.group)
        return facts

    @property
    def facts_in_payload(self) -> bool:
        """True when a processor call's facts travel in the exchange's payload
        (sparse and peer exchanges: ORed by the OR pass, no collective for
        them); the dense exchange sums them with an all_reduce."""
        return self.exchange in ("sparse", "peer")

    def stage(self, lo, hi, bits, vocab: int, facts=None) -> bool:
        """The peer exchange's pack (with the call's facts in the payload when
        given).  Without ``facts`` it is issued before the facts all_reduce, so
        that that collective is the exchange's barrier: True when staged that
        way."""
        if self.group is None or self.exchange != "peer":
            return False
        B = lo.numel()
        if self._peer is None or self._peer.rows < B or self._peer.vocab != vocab:
            self.close()
            self._peer = PeerExchange(self.group, B, vocab, lo.device, barrier=self.peer_barrier, spins=self.spins)
        self._peer.check()
        self.shard.shard_pack(lo, hi, bits, vocab, payload=self._peer.payload(), facts=facts)
        self._staged = True
        return facts is None and self.peer_barrier == "collective"

    def check_exchange(self):
        """Raise PeerBarrierTimeout if a peer-exchange step has timed out (no
        synchronisation: a host read; the processors call it after the wait
        they make anyway)."""
        if self._peer is not None:
            self._peer.check()

    def close(self):
        """Release the peer exchange's mappings (collective: every rank calls it);
        raises PeerBarrierTimeout if one of its steps timed out."""
        if self._peer is not None:
            px, self._peer = self._peer, None
            px.close()

    def or_bits(self, lo, hi, bits, vocab: int, staged: bool = False, facts=None):
        """OR of every rank's packed allowed bits (int32 [B, W]) -> int32 [B, W].
        ``staged``: stage() packed this step's payload before a collective
        every rank issued after it (the peer exchange's barrier).  ``facts``
        (int32 [3, B], sparse / peer exchanges): the call's facts ride in the
        payload (stage() packed them when it ran) and their OR over the ranks
        is returned too -> (words, facts_or)."""
        if self.group is None:
            return bits if facts is None else (bits, (facts != 0).to(facts.dtype))
        import torch
        import torch.distributed as dist

        B, W = lo.numel(), (vocab + 31) // 32
        fo = None
        if facts is not None:
            if not self.facts_in_payload:
                raise ValueError("or_bits: the dense exchange does not carry facts (sum_facts)")
            fo = torch.empty((3, B), dtype=torch.int32, device=lo.device)
        if self.exchange == "peer":
            if not self._staged:
                self.stage(lo, hi, bits, vocab, facts=facts)
                staged = False          # packed just now: no collective has run since
            self._staged = False
            w = self._peer(self._peer.payload(), B, vocab, self.shift, unpack=False, barrier_done=staged, facts_out=fo)
            return w if fo is None else (w, fo)
        if self.exchange == "sparse":
            self._payload = self.shard.shard_pack(lo, hi, bits, vocab, payload=self._payload, facts=facts)
            if self._xchg is None:
                self._xchg = SparseExchange(self.group)
            w = self._xchg(self._payload, B, vocab, self.shift, unpack=False, facts_out=fo)
            return w if fo is None else (w, fo)
        world = dist.get_world_size(self.group)
        mine = bits[:, :W].contiguous()
        if self._parts is None or self._parts.shape != (world, B, W):
            self._parts = torch.empty((world, B, W), dtype=torch.int32, device=bits.device)
        dist.all_gather_into_tensor(self._parts, mine, group=self.group)
        return or_bits(self._parts, vocab, unpack=False)

    # ---- the processors' host path over the shards (see the class docstring)
    def check_patterns(self, patterns):
        """HaloExceeded if a pattern is longer than the halo allows."""
        if self.halo is None or not patterns:
            return
        longest = max(len(p) for p in patterns)
        if longest > self.halo - 1:
            raise HaloExceeded(f"a pattern of {longest} tokens needs a halo of >= {longest + 1}; the shards were "
                               f"built with {self.halo}")

    def get_range_batch(self, patterns, shift: int = 10, starts=None):
        """get_range of every pattern on this rank's SHARD (shard-local (lo, hi):
        only its emptiness and the allowed bits it yields are global facts)."""
        return self.shard.get_range_batch(patterns, shift, starts=starts)

    def sum_counts(self, counts):
        """Per-pattern counts summed over the ranks (all_reduce SUM): zero exactly
        when the unsharded count is zero (halo duplicates inflate the rest)."""
        if self.group is None or not len(counts):
            return list(counts)
        import torch
        import torch.distributed as dist

        t = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=torch.device("cuda", self.device))
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.tolist()

    def allowed_mask(self, lo, hi, vocab: int, shift: int, out=None, packed: bool = False):
        """The allowed tokens of the shard-local ranges (lo, hi), ORed over the
        ranks -> int32 [B, ceil(V/32)] words (packed) or uint8 [B, V]: the
        unsharded index's mask of the same patterns."""
        bits = self.shard.allowed_mask(lo, hi, vocab, shift, packed=True)
        words = self.or_bits(lo, hi, bits, vocab)
        if packed:
            if out is not None:
                out.copy_(words)
                return out
            return words
        import torch

        W = (vocab + 31) // 32
        u8 = unpack_bits(words[:, :W].contiguous().view(torch.uint8), vocab)
        if out is not None:
            out.copy_(u8)
            return out
        return u8

    def size(self) -> int:
        return self.shard.size()


def payload_facts_at(B: int) -> int:
    """Word offset of a payload's facts area (after [4 words] desc[B] off[B], padded to 4)."""
    return 4 + ((2 * B + 3) & ~3)


def payload_header_words(B: int) -> int:
    """Words of a payload's header (csrc/fmidx_internal.h payload_header_words): the
    descriptors, then the facts area (3B words, padded to 4)."""
    return payload_facts_at(B) + ((3 * B + 3) & ~3)


def payload_capacity(B: int, vocab: int) -> int:
    """Worst-case uint32 words of a sparse-exchange payload of B rows."""
    from .fm_index import payload_capacity as _cap

    return _cap(B, vocab)


class SparseExchange:
    """The sparse exchange of one rank, per step: all_gather of the payload
    sizes, all_gather of the payloads, the OR pass.  The payload all_gather
    needs its size on the host, and reading the sizes there stalls the stream
    (the GPU then idles while the host enqueues the rest of the step).  So the
    payload gather and the OR pass are issued speculatively, BEFORE the sizes
    are read, with ``slack`` x the largest size of the last ``history`` steps;
    only when a rank's payload turns out larger (every rank sees the same
    sizes, so every rank takes the same decision) are they issued again with
    the real size.  Exact either way: a payload is read only up to its own
    header's size, and a gather at least that large holds all of it."""

    def __init__(self, group=None, slack: float = 1.25, history: int = 8):
        self.group = group
        self.slack = slack
        self.history = history
        self._max = []          # largest payload (words) of the recent steps (of this batch size)
        self._B = None
        self.words = []         # words every rank shipped, per step
        self.respecified = 0    # steps whose speculative size was too small

    def _gather(self, payload, m: int):
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        mine = payload[:m]
        if mine.numel() < m:                  # a host payload is exactly its size
            mine = torch.cat([mine, torch.zeros(m - mine.numel(), dtype=mine.dtype, device=mine.device)])
        parts = torch.empty(world * m, dtype=torch.int32, device=payload.device)
        dist.all_gather_into_tensor(parts, mine.contiguous(), group=self.group)
        return parts.view(world, m)

    def __call__(self, payload, B: int, vocab: int, shift: int, out=None, unpack: bool = True, facts_out=None):
        import torch
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        used = payload[:1].to(torch.int64)
        sizes = torch.empty(world, dtype=torch.int64, device=payload.device)
        dist.all_gather_into_tensor(sizes, used, group=self.group)
        guess = 0
        if B != self._B:                      # sizes of another batch size say nothing about this one
            self._max, self._B = [], B
        if self._max:
            # the same value on every rank (the sizes were gathered), never above a payload's capacity
            # nor below its header
            guess = min(payload_capacity(B, vocab),
                        max(payload_header_words(B), (int(max(self._max) * self.slack) + 3) & ~3))
            res = or_payloads(self._gather(payload, guess), B, vocab, shift, out=out, unpack=unpack, facts_out=facts_out)
        words = [int(x) for x in sizes.tolist()]
        m = max(words)
        self.words.append(words)
        self._max = (self._max + [m])[-self.history:]
        if guess and m <= guess:
            return res
        if guess:
            self.respecified += 1
        return or_payloads(self._gather(payload, m), B, vocab, shift, out=out, unpack=unpack, facts_out=facts_out)


class PeerBarrierTimeout(RuntimeError):
    """The flag barrier of a peer exchange timed out: some rank did not post
    its payload within the spin bound, so the OR pass of that step read
    payloads that may be stale or half-written.  Masks must be exact or
    absent: every later call of the exchange raises this too (the step's
    output was already returned -- the error is read without a per-step
    synchronisation, at the next call and at close())."""


class FmPeerStep(ctypes.Structure):
    """fm_peer_step (include/fmidx.h): one flag-barrier step's fixed buffers."""
    _fields_ = [("d_lo", ctypes.c_void_p), ("d_hi", ctypes.c_void_p), ("m", ctypes.c_uint64),
                ("d_payload", ctypes.c_void_p), ("d_payload_alt", ctypes.c_void_p), ("cap_words", ctypes.c_uint64),
                ("d_step", ctypes.c_void_p), ("d_flag_ptrs", ctypes.c_void_p), ("world", ctypes.c_uint64),
                ("d_done", ctypes.c_void_p), ("d_part_ptrs", ctypes.c_void_p), ("nparts", ctypes.c_uint64),
                ("d_flags", ctypes.c_void_p), ("spins", ctypes.c_uint32), ("err", ctypes.c_void_p),
                ("d_out", ctypes.c_void_p), ("ld_out", ctypes.c_uint64), ("unpack", ctypes.c_int32),
                ("vocab", ctypes.c_uint64), ("shift", ctypes.c_int64), ("reset_below", ctypes.c_int64)]


assert ctypes.sizeof(FmPeerStep) == 168 and FmPeerStep.reset_below.offset == 160   # api.cpp asserts the same


class PeerExchange:
    """The sparse exchange with no gather and no host read: every rank packs
    into one of two payload buffers of its own (double-buffered by step
    parity), whose IPC handles the ranks swapped once at construction
    (fm_ipc_handle / fm_ipc_open: the peers' buffers mapped over xGMI); after
    a stream-ordered barrier, ONE launch (fm_shard_or_rows_peers) reads every
    rank's payload in place and ORs them.

    ``barrier``: "collective" -- a one-element all_reduce issued after the
    pack (RCCL runs it after the rank's pack and completes it only when every
    rank's has run, so the OR that follows on the stream sees every payload;
    the processors pass ``barrier_done`` when their facts all_reduce, issued
    after the pack, already is one); "flags" (the default) -- no collective at
    all: after its pack every rank advances its device step counter and stores
    the new value into its word of every rank's flag array (fm_peer_signal,
    a system-scope release, then system-scope stores over xGMI) and the OR pass
    first waits for all of its own words (fm_shard_or_rows_peers_wait, then a
    system-scope acquire).  The step number and the buffer parity live on the
    device, so a step (decode + signal + OR) captured once into a HIP graph
    replays for every decode step.  The wait is bounded by ``spins`` polls
    (None: the library's 2^20, ~0.1-1 s); a step that times out is recorded in
    an error word in coherent host memory and the NEXT call (or close())
    raises PeerBarrierTimeout -- no per-step synchronisation; "host" --
    synchronize + group barrier (gloo; ranks sharing a GPU, where RCCL refuses
    to run).  Two buffers are enough: a rank packs buffer k again two steps
    later, after a barrier that every rank entered only after its OR of buffer
    k had been issued before it on its stream.  ``capacity_rows``: the largest
    batch the buffers hold (payload_capacity words each)."""

    def __init__(self, group, capacity_rows: int, vocab: int, device, barrier: str = "flags",
                 spins: Optional[int] = None):
        import torch
        import torch.distributed as dist
        from ctypes import byref, c_uint8, c_uint64, c_void_p

        from ._lib import check, lib

        if barrier not in ("collective", "host", "flags"):
            raise ValueError(barrier)
        self.group, self.barrier_mode, self.vocab = group, barrier, vocab
        self.spins = int(spins or 0)
        if not 0 <= self.spins < (1 << 32):
            raise ValueError("spins: 0 .. 2^32 - 1 polls")
        self.device = torch.device(device)
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world > 64:
            raise ValueError("PeerExchange: at most 64 ranks (the OR pass stages one part per lane of a wave)")
        self.rows = capacity_rows
        self.cap = payload_capacity(capacity_rows, vocab)
        self.bufs = [torch.zeros(self.cap, dtype=torch.int32, device=self.device) for _ in range(2)]
        # the flag barrier's words (one per rank) and this rank's step counter, shared like the payloads
        self.flags = torch.zeros(max(64, self.world), dtype=torch.int32, device=self.device)
        self.ctr = torch.zeros(1, dtype=torch.int32, device=self.device)
        # the fused signal's workgroup counts (csrc/decode.hip: 9 counters, 32 words apart)
        self.done = torch.zeros(9 * 32, dtype=torch.int32, device=self.device)
        # its error word: coherent host memory the OR pass stores into on a timeout
        ep = c_void_p()
        check(lib().fm_host_mapped_alloc(4, byref(ep)), "host_mapped_alloc")
        self._err_ptr = ep.value
        self._err_word = ctypes.c_int32.from_address(self._err_ptr)
        self._failed = 0
        self._skip_signal = 0        # tests: steps whose signal posts nothing (a rank that falls behind)
        self._step_key = None        # fm_peer_flags_step's struct, per (index, state, output)
        torch.cuda.synchronize(self.device)
        mine = []
        for b in self.bufs + [self.flags]:
            hd = (c_uint8 * 64)()
            off = c_uint64(0)
            check(lib().fm_ipc_handle(c_void_p(b.data_ptr()), hd, byref(off)), "ipc_handle")
            mine.append((bytes(hd), int(off.value)))
        every = [None] * self.world
        dist.all_gather_object(every, mine, group=group)
        self._opened = []
        table = [[0] * self.world for _ in range(3)]   # payload buffer 0, buffer 1, flag array
        try:
            for r, hs in enumerate(every):
                for k, (hd, off) in enumerate(hs):
                    if r == self.rank:
                        table[k][r] = (self.bufs + [self.flags])[k].data_ptr()
                        continue
                    base = c_void_p()
                    check(lib().fm_ipc_open((c_uint8 * 64).from_buffer_copy(hd), byref(base)), f"ipc_open (rank {r})")
                    self._opened.append(base.value)
                    table[k][r] = base.value + off
        except Exception:
            self._unmap()
            raise
        # [2, P]: buffer 0's addresses, then buffer 1's (the flag barrier's pass picks the row by
        # the device counter's parity; the other barriers pass the row of the host step)
        self.ptab = torch.tensor(table[:2], dtype=torch.int64, device=self.device)
        # this rank's word in every rank's flag array
        self.signal_to = torch.tensor([a + 4 * self.rank for a in table[2]], dtype=torch.int64, device=self.device)
        self._tok = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.step = 0

    def payload(self):
        """This step's payload buffer (pack into it, then call)."""
        return self.bufs[self.step % 2]

    def check(self):
        """Raise PeerBarrierTimeout if a flag-barrier step has timed out (a read
        of host memory: no synchronisation; a pass still running is seen at a
        later call)."""
        v = self._failed or (self._err_word.value if self._err_ptr else 0)
        if v:
            self._failed = v
            raise PeerBarrierTimeout(f"rank {self.rank}: the flag barrier of step {v & 0xFFFFFFFF} timed out "
                                     f"(a peer did not post its payload within the spin bound); that step's "
                                     f"OR was not exact and the exchange is unusable")

    def barrier(self):
        import torch
        import torch.distributed as dist

        if self.barrier_mode == "collective":
            dist.all_reduce(self._tok, group=self.group)
        else:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)

    def signal(self, stream=None):
        """fm_peer_signal: advance the device step counter and post it to every rank."""
        import torch
        from ctypes import c_void_p

        from ._lib import check, lib

        if stream is None:
            idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
            stream = torch._C._cuda_getCurrentRawStream(idx)   # (no Stream object per step)
        world = self.world
        if self._skip_signal:
            self._skip_signal -= 1
            world = 0
        check(lib().fm_peer_signal(c_void_p(self.signal_to.data_ptr()), world, c_void_p(self.ctr.data_ptr()),
                                   c_void_p(stream)), "peer_signal")

    def _fused_step(self, index, tokens, lo, hi, vocab, shift, out, unpack, reset_below, sync):
        """fm_peer_flags_step: the struct of this step's fixed buffers is built
        once per (index, state, output) and reused; per call only the tokens,
        the signal's world (the test hook) and the stream travel."""
        import torch
        from ctypes import addressof, c_void_p

        from ._lib import check, lib

        B = lo.numel()
        ld = out.stride(0) * out.element_size()
        key = (index._h.value if hasattr(index._h, "value") else index._h, lo.data_ptr(), hi.data_ptr(), B,
               out.data_ptr(), ld, bool(unpack), int(vocab), int(shift), int(reset_below))
        if self._step_key != key:
            W = (int(vocab) + 31) // 32
            want = (torch.uint8, int(vocab)) if unpack else (torch.int32, W)
            if not (out.dim() == 2 and out.stride(1) == 1 and out.device == self.device and out.dtype == want[0]
                    and out.shape[0] >= B and out.shape[1] >= want[1]):
                raise ValueError(f"flags_step: out must be a row-contiguous {want[0]} [>= {B}, >= {want[1]}] "
                                 f"tensor on {self.device}")
            if not (lo.dtype == hi.dtype == torch.int64 and lo.is_contiguous() and hi.is_contiguous()
                    and hi.numel() == B and lo.device == hi.device == self.device):
                raise ValueError("flags_step: lo / hi must be contiguous int64 tensors of one length on the device")
            st = FmPeerStep(d_lo=lo.data_ptr(), d_hi=hi.data_ptr(), m=B, d_payload=self.bufs[0].data_ptr(),
                            d_payload_alt=self.bufs[1].data_ptr(), cap_words=self.cap, d_step=self.ctr.data_ptr(),
                            d_flag_ptrs=self.signal_to.data_ptr(), world=self.world, d_done=self.done.data_ptr(),
                            d_part_ptrs=self.ptab.data_ptr(), nparts=self.ptab.shape[-1],
                            d_flags=self.flags.data_ptr(), spins=self.spins, err=self._err_ptr or None,
                            d_out=out.data_ptr(), ld_out=ld, unpack=1 if unpack else 0, vocab=int(vocab),
                            shift=int(shift), reset_below=int(reset_below))
            self._step_struct, self._step_key = st, key
            self._step_arg = c_void_p(addressof(st))
        if tokens.dtype != torch.int64 or tokens.numel() < B or tokens.device != self.device:
            raise ValueError(f"flags_step: tokens must be an int64 tensor of >= {B} ids on {self.device}")
        st = self._step_struct
        st.world = self.world
        if self._skip_signal:
            self._skip_signal -= 1
            st.world = 0
        stream = torch._C._cuda_getCurrentRawStream(self.device.index)
        rc = lib().fm_peer_flags_step(index._h, self._step_arg, c_void_p(tokens.data_ptr()), 1 if sync else 0,
                                      c_void_p(stream))
        if rc < 0:
            check(rc, "peer_flags_step")
        return out

    def flags_step(self, index, tokens, lo, hi, vocab: int, shift: int, out, unpack: bool = True,
                   reset_below: int = 0, sync=None):
        """One decode step with the flag barrier, as two stream-ordered
        launches and nothing else (capturable; a captured call replays for
        every step): the payload decode of ``index`` -- the state (lo, hi)
        updated in place, the payload buffer picked by the counter's parity,
        the signal fused into its last workgroup -- then the OR pass into
        ``out`` (an index without the fused form: three launches, the signal
        its own).  The caller counts executed steps
        in ``self.step`` (host parity = device parity, for payload()).  ``sync``
        (True / False; None = the separate launches): one C call
        (fm_peer_flags_step) for both launches, with True also the stream's
        synchronisation -- the error word is then current for check()."""
        if self.barrier_mode != "flags":
            raise ValueError("flags_step: the exchange's barrier is not the flag barrier")
        B = lo.numel()
        if B > self.rows or vocab != self.vocab:
            raise ValueError(f"PeerExchange holds {self.rows} rows of vocab {self.vocab}")
        if sync is not None and hasattr(index, "_h"):
            # both launches (and, with sync, the wait and the error word) in one C call
            return self._fused_step(index, tokens, lo, hi, vocab, shift, out, unpack, reset_below, sync)
        if hasattr(index, "decode_step_payload_signal"):
            # the signal fused into the decode kernel (its last workgroup posts the step): two launches
            world = self.world
            if self._skip_signal:
                self._skip_signal -= 1
                world = 0
            index.decode_step_payload_signal(tokens, lo, hi, self.bufs[0], self.bufs[1], self.ctr, self.signal_to,
                                             world, self.done, vocab, shift, reset_below=reset_below)
        else:
            index.decode_step_payload(tokens, lo, hi, lo, hi, self.bufs[0], vocab, shift, reset_below=reset_below,
                                      payload_alt=self.bufs[1], step=self.ctr)
            self.signal()
        return self.or_flags(B, vocab, shift, out=out, unpack=unpack)

    def or_flags(self, B: int, vocab: int, shift: int, out=None, unpack: bool = True, facts_out=None):
        """The flag barrier's OR pass of the step the counter names (its payload
        buffer by the counter's parity)."""
        return or_peer_payloads(self.ptab, self.cap, B, vocab, shift, out=out, unpack=unpack,
                                flags=(self.flags, self.ctr, self._err_ptr, self.spins), buffers=2,
                                facts_out=facts_out)

    def __call__(self, payload, B: int, vocab: int, shift: int, out=None, unpack: bool = True,
                 barrier_done: bool = False, facts_out=None):
        self.check()
        k = self.step % 2
        if payload.data_ptr() != self.bufs[k].data_ptr():
            raise ValueError("PeerExchange: pack into payload() of this step")
        if B > self.rows or vocab != self.vocab:
            raise ValueError(f"PeerExchange holds {self.rows} rows of vocab {self.vocab}")
        if self.barrier_mode == "flags":
            self.signal()
            out = self.or_flags(B, vocab, shift, out=out, unpack=unpack, facts_out=facts_out)
        else:
            if not barrier_done:
                self.barrier()
            out = or_peer_payloads(self.ptab[k], self.cap, B, vocab, shift, out=out, unpack=unpack,
                                   facts_out=facts_out)
        self.step += 1
        return out

    def errors(self) -> int:
        """The last step number whose flag barrier timed out (0: none), after a
        synchronisation of the device."""
        import torch

        torch.cuda.synchronize(self.device)
        return int(self._failed or (self._err_word.value if self._err_ptr else 0))

    def _unmap(self):
        from ctypes import c_void_p

        from ._lib import lib

        for base in self._opened:
            lib().fm_ipc_close(c_void_p(base))
        self._opened = []

    def close(self):
        """Unmap the peers' buffers once no rank reads any buffer (a
        synchronize + group barrier: no rank frees its buffers while a peer
        may still read them); raises PeerBarrierTimeout if a step timed out."""
        import torch
        import torch.distributed as dist
        from ctypes import c_void_p

        from ._lib import lib

        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)
        self._unmap()
        failed = self._failed or (self._err_word.value if self._err_ptr else 0)
        if self._err_ptr:
            lib().fm_host_mapped_free(c_void_p(self._err_ptr))
            self._err_ptr, self._err_word = 0, None
        if failed:
            self._failed = failed
            self.check()


def or_peer_payloads(ptrs, cap: int, B: int, vocab: int, shift: int, out=None, unpack: bool = True, flags=None,
                     buffers: int = 1, facts_out=None):
    """OR of the payloads at the device addresses ``ptrs`` (int64 [P], on the
    GPU that runs the pass; each payload ``cap`` words, in this process or a
    peer's buffer mapped by fm_ipc_open) -> uint8 [B, vocab] (unpack) or int32
    [B, ceil(vocab/32)] words (fm_shard_or_rows_peers).  ``flags`` = (flag
    words int32 [>= P], the step counter int32 [1], the error word's address,
    spins): the flag barrier first (fm_shard_or_rows_peers_wait); ``ptrs`` is
    then [2, P], the double buffer's two address rows (``buffers`` = 2).
    ``facts_out`` (int32 [3, B]): the OR of the payloads' facts areas
    (fm_shard_or_rows_peers_facts)."""
    import torch
    from ctypes import c_void_p

    from ._lib import check, lib

    W = (vocab + 31) // 32
    if not (ptrs.is_cuda and ptrs.dtype == torch.int64 and ptrs.dim() == buffers and ptrs.is_contiguous()):
        raise ValueError(f"ptrs: a contiguous int64 device tensor of {buffers} dimension(s)")
    if (flags is None) != (buffers == 1):
        raise ValueError("the flag barrier reads both payload buffers' address rows; the others one row")
    nparts = ptrs.shape[-1]
    if out is None:
        out = (torch.empty((B, vocab), dtype=torch.uint8, device=ptrs.device) if unpack
               else torch.empty((B, W), dtype=torch.int32, device=ptrs.device))
    assert out.stride(1) == 1 and out.device == ptrs.device
    ld = out.stride(0) * out.element_size()
    stream = torch._C._cuda_getCurrentRawStream(ptrs.device.index)
    if facts_out is not None:
        _check_facts(facts_out, B, ptrs.device)
        fw, ctr, err_ptr, spins = flags if flags is not None else (None, None, None, 0)
        if fw is not None and fw.numel() < nparts:
            raise ValueError("flag words: one per part")
        check(lib().fm_shard_or_rows_peers_facts(
            c_void_p(ptrs.data_ptr()), nparts, int(cap), B, vocab, int(shift), c_void_p(out.data_ptr()), ld,
            1 if unpack else 0, c_void_p(fw.data_ptr()) if fw is not None else None,
            c_void_p(ctr.data_ptr()) if ctr is not None else None, int(spins), c_void_p(err_ptr) if err_ptr else None,
            c_void_p(facts_out.data_ptr()), c_void_p(stream)), "shard_or_rows_peers_facts")
        return out
    if flags is not None:
        fw, ctr, err_ptr, spins = flags
        if fw.numel() < nparts:
            raise ValueError("flag words: one per part")
        check(lib().fm_shard_or_rows_peers_wait(c_void_p(ptrs.data_ptr()), nparts, int(cap), B, vocab,
                                                int(shift), c_void_p(out.data_ptr()), ld, 1 if unpack else 0,
                                                c_void_p(fw.data_ptr()), c_void_p(ctr.data_ptr()), int(spins),
                                                c_void_p(err_ptr), c_void_p(stream)), "shard_or_rows_peers_wait")
        return out
    check(lib().fm_shard_or_rows_peers(c_void_p(ptrs.data_ptr()), nparts, int(cap), B, vocab, int(shift),
                                       c_void_p(out.data_ptr()), ld, 1 if unpack else 0, c_void_p(stream)),
          "shard_or_rows_peers")
    return out


def or_payloads(parts, B: int, vocab: int, shift: int, out=None, unpack: bool = True, facts_out=None):
    """OR of the ranks' sparse-exchange payloads ``parts`` (int32 [P, stride])
    -> uint8 [B, vocab] (unpack) or int32 [B, ceil(vocab/32)] words.  GPU:
    fm_shard_or_rows(_facts); CPU tensors (gloo tests): the same format read
    with torch ops (or_payloads_host).  ``facts_out`` (int32 [3, B]): the OR of
    the payloads' facts areas."""
    import torch
    from ctypes import c_void_p

    from ._lib import check, lib

    if not parts.is_cuda:
        return or_payloads_host(parts, B, vocab, shift, unpack=unpack, facts_out=facts_out)
    P, stride = parts.shape
    W = (vocab + 31) // 32
    if out is None:
        out = (torch.empty((B, vocab), dtype=torch.uint8, device=parts.device) if unpack
               else torch.empty((B, W), dtype=torch.int32, device=parts.device))
    assert parts.dtype == torch.int32 and parts.is_contiguous() and out.stride(1) == 1
    ld = out.stride(0) * out.element_size()
    stream = torch._C._cuda_getCurrentRawStream(parts.device.index)
    if facts_out is not None:
        _check_facts(facts_out, B, parts.device)
        check(lib().fm_shard_or_rows_facts(c_void_p(parts.data_ptr()), P, stride, B, vocab, int(shift),
                                           c_void_p(out.data_ptr()), ld, 1 if unpack else 0,
                                           c_void_p(facts_out.data_ptr()), c_void_p(stream)), "shard_or_rows_facts")
        return out
    check(lib().fm_shard_or_rows(c_void_p(parts.data_ptr()), P, stride, B, vocab, int(shift), c_void_p(out.data_ptr()),
                                 ld, 1 if unpack else 0, c_void_p(stream)), "shard_or_rows")
    return out


def _check_facts(f, B: int, device):
    import torch

    if not (f.dtype == torch.int32 and f.is_contiguous() and f.numel() == 3 * B and f.device == device):
        raise ValueError(f"facts: a contiguous int32 [3, {B}] tensor on {device}")


_PAYLOAD_MAGIC = 0x58534D46


def pack_payload_host(lo, hi, bwt, bits_words, vocab: int, facts=None):
    """The sparse-exchange payload (csrc/shard.hip's layout) built on the host
    from a shard's BWT (int array) and its packed rows (int32 [B, >= W]) --
    for CPU indexes (gloo tests); the GPU path is fm_shard_pack(_facts).
    ``facts``: int [3, B] for the facts area (zeros without)."""
    import torch

    lo = np.asarray(lo, dtype=np.int64)
    hi = np.minimum(np.asarray(hi, dtype=np.int64), len(bwt))
    B = lo.size
    W = (vocab + 31) // 32
    H = payload_header_words(B)
    bw = np.asarray(bits_words, dtype=np.int64).astype(np.uint32)
    desc, off, data = np.zeros(B, dtype=np.uint32), np.zeros(B, dtype=np.uint32), []
    at = H
    for b in range(B):
        w = max(0, int(hi[b] - lo[b]))
        dense = w >= W
        row = bw[b, :W] if dense else np.asarray(bwt[lo[b]:lo[b] + w], dtype=np.uint32)
        pad = (-row.size) % 4
        desc[b] = row.size | (0x80000000 if dense else 0)
        off[b] = at
        data.append(np.concatenate([row, np.zeros(pad, dtype=np.uint32)]))
        at += row.size + pad
    head = np.zeros(H, dtype=np.uint32)
    head[:4] = [at, B, W, _PAYLOAD_MAGIC]
    head[4:4 + B] = desc
    head[4 + B:4 + 2 * B] = off
    if facts is not None:
        F = payload_facts_at(B)
        head[F:F + 3 * B] = (np.asarray(facts).reshape(3, B) != 0).astype(np.uint32).reshape(-1)
    out = np.concatenate([head] + data)
    return torch.from_numpy(out.view(np.int32).copy())


def or_payloads_host(parts, B: int, vocab: int, shift: int, unpack: bool = True, facts_out=None):
    """The OR pass on the host (gloo tests).  ``facts_out`` (a torch int32 [3, B]
    tensor): the OR over the parts of their facts areas is written into it."""
    import torch

    W = (vocab + 31) // 32
    bits = np.zeros((B, W * 32), dtype=np.uint8)
    F = payload_facts_at(B)
    fo = np.zeros((3, B), dtype=np.int32)
    for p in parts.cpu().numpy().view(np.uint32):
        assert int(p[3]) == _PAYLOAD_MAGIC and int(p[1]) == B and int(p[2]) == W
        fo |= (p[F:F + 3 * B].reshape(3, B) != 0).astype(np.int32)
        for b in range(B):
            d, o = int(p[4 + b]), int(p[4 + B + b])
            cnt = d & 0x7FFFFFFF
            if o + ((cnt + 3) & ~3) > p.size:   # past a short gather's end: read as empty (fm_shard_or_rows too)
                continue
            if d >> 31:
                bits[b] |= np.unpackbits(p[o:o + W].view(np.uint8), bitorder="little")
            else:
                tok = p[o:o + cnt].astype(np.int64) - shift
                tok = tok[(tok >= 0) & (tok < vocab)]
                bits[b, tok] = 1
    if facts_out is not None:
        facts_out.copy_(torch.from_numpy(fo))
    if unpack:
        return torch.from_numpy(bits[:, :vocab].copy())
    return torch.from_numpy(np.packbits(bits, axis=1, bitorder="little").view(np.int32).copy())


def or_bits(parts, vocab: int, out=None, unpack: bool = True):
    """OR of the shards' bit-packed allowed rows (fm_or_bits, csrc/shard.hip):
    ``parts`` int32 [P, B, W] on the GPU -> uint8 [B, vocab] (unpack) or the
    ORed int32 [B, W] words."""
    import torch
    from ctypes import c_void_p

    from ._lib import check, lib

    P, B, W = parts.shape
    assert parts.is_cuda and parts.dtype == torch.int32 and parts.is_contiguous()
    if out is None:
        out = (torch.empty((B, vocab), dtype=torch.uint8, device=parts.device) if unpack
               else torch.empty((B, W), dtype=torch.int32, device=parts.device))
    want = (B, vocab) if unpack else (B, W)
    if tuple(out.shape) != want or out.stride(1) != 1 or out.dtype != (torch.uint8 if unpack else torch.int32):
        raise ValueError(f"or_bits: out must be a row-major {'uint8' if unpack else 'int32'} {want}, "
                         f"got {out.dtype} {tuple(out.shape)} strides {out.stride()}")
    ld = out.stride(0) * out.element_size()
    stream = torch._C._cuda_getCurrentRawStream(parts.device.index)
    check(lib().fm_or_bits(c_void_p(parts.data_ptr()), P, B * W, B, W, vocab, c_void_p(out.data_ptr()), ld,
                           1 if unpack else 0, c_void_p(stream)), "or_bits")
    return out


def pack_bits(mask_u8):
    """uint8 0/1 [B, V] -> uint8 [B, ceil(V/8)] little-endian bit order."""
    import torch

    B, V = mask_u8.shape
    pad = (-V) % 8
    m = mask_u8
    if pad:
        m = torch.cat([m, torch.zeros((B, pad), dtype=m.dtype, device=m.device)], 1)
    w = (torch.ones(8, dtype=torch.uint8, device=m.device) << torch.arange(8, dtype=torch.uint8, device=m.device))
    return (m.view(B, -1, 8) * w).sum(2).to(torch.uint8)


def unpack_bits(packed, vocab: int):
    import torch

    B = packed.shape[0]
    w = (torch.ones(8, dtype=torch.uint8, device=packed.device) << torch.arange(8, dtype=torch.uint8,
                                                                                 device=packed.device))
    bits = (packed.unsqueeze(2) & w).ne(0).to(torch.uint8).view(B, -1)
    return bits[:, :vocab].contiguous()


__all__ = ["shard_docs", "peer_capable", "host_identity", "halo_tokens", "shard_corpus", "shard_text_device", "ShardedDecoder", "HaloExceeded",
           "ShardedIndex",
           "or_bits", "pack_bits", "unpack_bits", "payload_capacity", "or_payloads", "SparseExchange",
           "PeerExchange", "PeerBarrierTimeout", "or_peer_payloads", "pack_payload_host", "or_payloads_host",
           "payload_header_words", "payload_facts_at"]
