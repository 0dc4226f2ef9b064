"""Document-constrained logits processors on the MI355X engine.

Drop-in counterparts of the reference's in-process processors, same
constructor arguments and call semantics, bit-identical outputs:

* ``QwenIndexBasedLogitsProcessor``  -- document_constrained_generation_causal_qwen.py:7-214
* ``CausalIndexBasedLogitsProcessor`` -- document_constrained_generation_causal.py:7-180
* ``SeqIndexBasedLogitsProcessor``   -- document_constrained_generation_seq.py:6-123
* ``VllmIndexBasedLogitsProcessor``  -- document_constrained_generation_vllm.py:6-137

What changes is how a step executes.  The reference walks rows in Python,
makes one SWIG call per pattern token (index.py:109-112) two or three times
per row, fans distinct_count_multi out over threads, copies each row's
distinct list host->device and builds the mask with ``torch.isin`` and two
index-puts per row.  Here a step is: the cheap per-row token bookkeeping in
Python (end marker, think marker, trailing n-gram rule, eos/pad rules), ONE
batched range search for all rows (``fm_get_range_batch``), ONE packed
allowed-token mask launch for all rows (``fm_allowed_mask_batch``) and ONE
fused epilogue that writes ``scores + mask`` (``fm_apply_boosts``) -- no
per-row device traffic.  The boost values are rounded to the scores dtype
exactly as torch rounds a Python float on assignment, and the add happens in
that dtype, so outputs match the reference bit for bit.
"""
from __future__ import annotations

import ctypes
import functools
import math
import os
from ctypes import c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p
from typing import List, Optional, Sequence

import numpy as np
import torch

from ._lib import check, lib

SHIFT = 10
FLAG_BITS, FLAG_UNIGRAM, FLAG_EOS, FLAG_SPECIAL = 1, 2, 4, 8
ROW_DTYPE = np.dtype([("base", "<f4"), ("v_dist", "<f4"), ("v_uni", "<f4"), ("v_eos", "<f4"),
                      ("flags", "<u4"), ("reserved", "<i4"), ("special", "<i8")])
_DTYPE_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


@functools.lru_cache(maxsize=4096)
def _round(x, dtype) -> float:
    """The value a Python number takes when index-put into a ``dtype`` tensor
    (the reference's ``mask[row, idx] = boost``), through the same setitem path.
    Memoised: a step asks for a few distinct values, but for every row."""
    t = torch.zeros(1, dtype=dtype)
    t[0] = x
    return float(t[0])


class _PrepConfig(ctypes.Structure):
    """fm_prep_config (include/fmidx.h)."""
    _fields_ = [("marker", c_int64 * 8), ("think", c_int64 * 2), ("sys", c_int64 * 4), ("eos", c_int64),
                ("pad", c_int64), ("stop_at_count", c_int64), ("min_new_tokens", c_int64), ("forced_bos", c_int64),
                ("shift", c_int64), ("marker_len", c_int32), ("num_beams", c_int32), ("flags", c_uint32),
                ("base", c_float), ("v_uni_full", c_float), ("v_uni_half", c_float), ("v_forced", c_float),
                ("skip", c_int32)]


assert ctypes.sizeof(_PrepConfig) == 192
PREP_THINK, PREP_SKIP_FIRST, PREP_EOS, PREP_EOS_ALL, PREP_UNI_HALF, PREP_HARD = 1, 2, 4, 8, 16, 32


def _boost_table(boost: float, lrf: float, dtype, n: int) -> List[float]:
    """BOOST * lrf ** k (the reference's Python float arithmetic, k < n)
    rounded like an index-put into ``dtype``; NaN where the reference's
    assignment raises instead -- ``lrf ** k`` is not a finite Python float
    (OverflowError) or the value does not fit ``dtype`` (torch's RuntimeError):
    rows needing such an entry take the host path, which raises the same."""
    out = []
    for k in range(n):
        try:
            out.append(_round(boost * (lrf ** k), dtype))
        except (OverflowError, RuntimeError):
            out.append(math.nan)
    return out


_CFG_ATTRS = ("eos_token_id", "pad_token_id", "stop_at_count", "min_new_tokens", "always_allow_eos",
              "forced_bos_token_id", "length_reward_factor", "BOOST", "_num_beams", "model_name")


def _config(proc, dtype) -> "_PrepConfig":
    """proc._prep_config(dtype), built once per dtype and attribute values
    (a call would otherwise rebuild the ctypes struct and round its boosts:
    ~10 us of a vLLM per-sequence call's host time)."""
    sig = (dtype, tuple(getattr(proc, "end_marker", ())), tuple(proc.force_decoding_from or ())) + \
        tuple(getattr(proc, a, None) for a in _CFG_ATTRS)
    cache = proc.__dict__.setdefault("_cfg_cache", {})
    c = cache.get(sig)
    if c is None:
        c = cache[sig] = proc._prep_config(dtype)
    return c


def _raw_stream(dev_index: int) -> int:
    """torch's current stream on the device as a raw hipStream_t (the C call
    behind torch.cuda.current_stream(...).cuda_stream, without building the
    Stream object)."""
    return torch._C._cuda_getCurrentRawStream(dev_index)


class SpeculativeCallError(RuntimeError):
    """FMIDX_PROC_STATUS=deferred: an earlier call returned the device path's
    output for an input whose reference result needs the host path."""


class _ProcessorArgs(ctypes.Structure):
    """fm_processor_args (include/fmidx.h)."""
    _fields_ = [("ids", c_void_p), ("B", c_uint64), ("L", c_uint64), ("ld", c_uint64), ("fdf", c_void_p),
                ("fdf_len", c_uint64), ("pow_tab", c_void_p), ("pow_len", c_uint64), ("prev_ids", c_void_p),
                ("prev_ld", c_uint64), ("prev_B", c_uint64), ("prev_state", c_void_p), ("rows", c_void_p),
                ("mask_lo", c_void_p), ("mask_hi", c_void_p), ("state", c_void_p), ("status", c_void_p),
                ("bits", c_void_p), ("bits_ld", c_uint64), ("dtype", c_int32), ("reserved", c_int32),
                ("scores", c_void_p), ("out", c_void_p), ("V", c_uint64), ("ld_scores", c_uint64),
                ("ld_out", c_uint64), ("unigram_bits", c_void_p), ("eos", c_int64), ("ids_copy", c_void_p),
                ("copy_ld", c_uint64), ("status_host", c_void_p), ("status_event", c_void_p)]


assert ctypes.sizeof(_ProcessorArgs) == 248


class _DeviceStep:
    """One soft-processor call on the device, ONE C call (fm_processor_call):
    the per-row bookkeeping + pattern ranges (csrc/process.hip), the packed
    allowed bits of the rows that need them, the fused epilogue, this call's
    input_ids kept for the next call and the status copied to pinned memory.
    Buffers persist across calls (the row state and the kept ids ping-pong
    between two sets), so a row whose pattern grew by one token costs ONE LF
    step and a call allocates only its output.  Returns None when a row does
    not have exactly one end marker at a common position (or a boost
    overflows): the caller then runs the host path, which reproduces the
    reference's behaviour for such inputs."""

    WAIT_STREAM = False    # measurement: wait for the whole call instead of the status event
    VERIFY_HARD = False    # measurement: hard-mask calls read their status too

    def __init__(self, core: "_BatchedCore", boost: float, lrf: float, fdf: Optional[List[int]]):
        self.core = core
        self.index = core.index
        self.dev = torch.device("cuda", self.index.device)
        self.boost = boost
        self.lrf = lrf
        self.fdf = torch.tensor(list(fdf or []) + [0], dtype=torch.int64, device=self.dev)
        self.fdf_len = len(fdf or [])
        self._pow = {}
        self.status = torch.zeros(4, dtype=torch.int32, device=self.dev)
        self.status_h = torch.zeros(4, dtype=torch.int32).pin_memory()
        self._status_np = self.status_h.numpy()
        self._args = _ProcessorArgs()
        self._B = -1
        self._bufs = None
        self._ids = [None, None]      # kept input_ids, ping-pong
        self._state = [None, None]
        self._cur = 0                 # the set the next call writes
        self._prev_ok = False         # the other set holds a valid previous call
        # The call's status is read after an event recorded right behind the row
        # bookkeeping (k_prep + the status copy), not after the whole call: the
        # mask and the epilogue are still running when the output is returned
        # (torch's stream order covers its consumers).  WAIT_STREAM = True
        # restores the full synchronize (measurement only: tools/bench_generate.py).
        self._ev = torch.cuda.Event()
        self._ev_ready = False
        self._wait_stream = type(self).WAIT_STREAM
        self._verify = type(self).VERIFY_HARD    # hard calls: read the status anyway
        # FMIDX_PROC_STATUS=deferred (opt-in, measurement of the wait's cost): a soft call returns
        # without waiting for its status; the status is checked at the next call (or check_pending())
        # and a call that needed the host path raises SpeculativeCallError there -- its output was
        # the device path's, not the reference's.  Default: every soft call waits (exact).
        self._deferred = os.environ.get("FMIDX_PROC_STATUS", "wait") == "deferred"
        self._pend = None
        self._pend_bufs = None

    def check_pending(self):
        """Deferred-status mode: raise if the last call needed the host path."""
        pend, self._pend = self._pend, None
        if pend is None:
            return
        ev, st = pend
        ev.synchronize()
        if st[0] != 0 or st[1] != st[2]:
            self._prev_ok = False
            raise SpeculativeCallError("a previous processor call's input needed the host path (end markers / "
                                       "boost overflow); with FMIDX_PROC_STATUS=deferred its output was the "
                                       "device path's")

    @property
    def prev_ids(self):
        """The previous call's input_ids as kept on the device (None after a
        host-path call or before the first call)."""
        return self._ids[1 - self._cur] if self._prev_ok else None

    def _pow_table(self, dtype, need: int):
        t = self._pow.get(dtype)
        if t is None or t.numel() < need:
            n = max(need, 2 * (t.numel() if t is not None else 256))
            t = torch.tensor(_boost_table(self.boost, self.lrf, dtype, n), dtype=torch.float32, device=self.dev)
            self._pow[dtype] = t
        return t

    def _buffers(self, B: int, V: int):
        words = (V + 31) // 32
        if self._bufs is None or self._B != B or self._bufs["words"] < words:
            dev = self.dev
            self._bufs = {"rows": torch.empty(B * ROW_DTYPE.itemsize, dtype=torch.uint8, device=dev),
                          "mlo": torch.empty(B, dtype=torch.int64, device=dev),
                          "mhi": torch.empty(B, dtype=torch.int64, device=dev),
                          "bits": torch.empty((B, words), dtype=torch.int32, device=dev), "words": words}
            self._state = [torch.empty((4, B), dtype=torch.int64, device=dev) for _ in range(2)]
            self._B = B
            self._prev_ok = False
        return self._bufs

    def __call__(self, input_ids, scores, cfg: _PrepConfig, wait: bool = True):
        """wait=False (the hard-mask variants): the call's status is fixed by
        its inputs -- no end marker to find, every boost 0 -- so the device
        path always holds and the host neither copies nor waits for it: the call
        only enqueues work (vLLM V0 calls one clone per sequence per step)."""
        if not wait and not (cfg.flags & PREP_HARD):
            raise ValueError("wait=False is only valid for hard-mask (PREP_HARD) calls: a soft call's status "
                             "(end markers, boost overflow) depends on its input and must be read")
        dev = self.dev
        ids = input_ids if (input_ids.device == dev and input_ids.dtype == torch.int64
                            and input_ids.is_contiguous()) else input_ids.to(dev, torch.int64).contiguous()
        if ids.dim() != 2:
            return None
        B, Lt = ids.shape
        if B != scores.shape[0] or B % max(1, cfg.num_beams):
            return None
        dtype = scores.dtype
        if dtype not in _DTYPE_CODE:
            raise TypeError(f"unsupported scores dtype {dtype}")
        V = scores.shape[1]
        src = scores if (scores.device == dev and scores.is_contiguous()) else scores.to(dev).contiguous()
        out = torch.empty_like(src)
        pow_t = self._pow_table(dtype, Lt + 1)
        bufs = self._buffers(B, V)
        cur, oth = self._cur, 1 - self._cur
        keep = self._ids[cur]
        if keep is None or keep.shape[0] != B or keep.shape[1] < Lt:
            keep = torch.empty((B, max(Lt + 64, 2 * (keep.shape[1] if keep is not None else 0))), dtype=torch.int64,
                               device=dev)
            self._ids[cur] = keep
        prev = self._ids[oth] if self._prev_ok else None
        a = self._args
        a.ids, a.B, a.L, a.ld = ids.data_ptr(), B, Lt, Lt
        a.fdf, a.fdf_len = self.fdf.data_ptr(), self.fdf_len
        a.pow_tab, a.pow_len = pow_t.data_ptr(), pow_t.numel()
        if prev is not None:
            a.prev_ids, a.prev_ld, a.prev_B, a.prev_state = prev.data_ptr(), prev.stride(0), prev.shape[0], \
                self._state[oth].data_ptr()
        else:
            a.prev_ids, a.prev_ld, a.prev_B, a.prev_state = None, 0, 0, None
        a.rows, a.mask_lo, a.mask_hi = bufs["rows"].data_ptr(), bufs["mlo"].data_ptr(), bufs["mhi"].data_ptr()
        a.state, a.status = self._state[cur].data_ptr(), self.status.data_ptr()
        a.bits, a.bits_ld = bufs["bits"].data_ptr(), bufs["words"]
        a.dtype = _DTYPE_CODE[dtype]
        a.scores, a.out, a.V, a.ld_scores, a.ld_out = src.data_ptr(), out.data_ptr(), V, src.stride(0), out.stride(0)
        a.unigram_bits = self.core.unigram_bits(V, dev).data_ptr()
        a.eos = int(cfg.eos)
        a.ids_copy, a.copy_ld = keep.data_ptr(), keep.stride(0)
        if self._deferred:
            self.check_pending()
        wait = wait or self._verify or B == 0
        if wait and self._deferred and B and not (cfg.flags & PREP_HARD):
            if self._pend_bufs is None:
                self._pend_bufs = [(torch.cuda.Event(), torch.zeros(4, dtype=torch.int32).pin_memory())
                                   for _ in range(2)]
            ev, st = self._pend_bufs[self._cur]
            ev.record(torch.cuda.current_stream(dev))      # creates the event; re-recorded by the call
            a.status_host, a.status_event = st.data_ptr(), ev.cuda_event
            check(lib().fm_processor_call(self.index._h, ctypes.byref(cfg), ctypes.byref(a),
                                          c_void_p(_raw_stream(dev.index))), "processor_call")
            self._pend = (ev, st.numpy())
            self._cur, self._prev_ok = oth, True
            return out if out.device == scores.device else out.to(scores.device)
        if wait:
            a.status_host = self.status_h.data_ptr()
            if not self._ev_ready:          # torch creates the event at its first record
                self._ev.record(torch.cuda.current_stream(dev))
                self._ev_ready = True
            a.status_event = self._ev.cuda_event
        else:
            a.status_host = a.status_event = None
        check(lib().fm_processor_call(self.index._h, ctypes.byref(cfg), ctypes.byref(a),
                                      c_void_p(_raw_stream(dev.index))), "processor_call")
        if not wait:
            self._cur, self._prev_ok = oth, True
            return out if out.device == scores.device else out.to(scores.device)
        if self._wait_stream:
            torch.cuda.current_stream(dev).synchronize()
        else:
            self._ev.synchronize()
        st = self._status_np
        if st[0] != 0 or st[1] != st[2]:
            self._prev_ok = False
            return None
        self._cur, self._prev_ok = oth, True
        return out if out.device == scores.device else out.to(scores.device)


class _ShardedDeviceStep(_DeviceStep):
    """A processor call over a doc-range shard (``fmidx.sharding.ShardedIndex``):
    fm_processor_shard_prep on this rank's shard (the row bookkeeping, the
    shard's ranges, the index-dependent facts and the shard's allowed bits),
    the exchange (facts summed over the ranks, bits ORed -- the sparse or the
    dense exchange), then fm_processor_shard_finish (the decisions from the
    summed facts, the epilogue with the ORed bits).  Every rank returns the
    same output, equal bit for bit to the unsharded processor's (SURVEY §8e:
    masks, emptiness and count([last]) > 0 are exact under an OR).  ``prep`` /
    ``finish`` are separate so that one process can drive several shards
    (tests, the one-GPU rehearsal)."""

    def __init__(self, core: "_BatchedCore", boost: float, lrf: float, fdf: Optional[List[int]]):
        super().__init__(core, boost, lrf, fdf)
        self.sidx = core.index
        self.index = core.index.shard

    def prep(self, input_ids, scores, cfg: _PrepConfig):
        dev = self.dev
        ids = input_ids if (input_ids.device == dev and input_ids.dtype == torch.int64
                            and input_ids.is_contiguous()) else input_ids.to(dev, torch.int64).contiguous()
        if ids.dim() != 2:
            return None
        B, Lt = ids.shape
        if B != scores.shape[0] or B % max(1, cfg.num_beams):
            return None
        dtype = scores.dtype
        if dtype not in _DTYPE_CODE:
            raise TypeError(f"unsupported scores dtype {dtype}")
        V = scores.shape[1]
        src = scores if (scores.device == dev and scores.is_contiguous()) else scores.to(dev).contiguous()
        out = torch.empty_like(src)
        pow_t = self._pow_table(dtype, Lt + 1)
        bufs = self._buffers(B, V)
        if "facts" not in bufs or bufs["facts"].shape[1] != B:
            bufs["facts"] = torch.empty((3, B), dtype=torch.int32, device=dev)
            bufs["rowcase"] = torch.empty(B, dtype=torch.int32, device=dev)
        cur, oth = self._cur, 1 - self._cur
        keep = self._ids[cur]
        if keep is None or keep.shape[0] != B or keep.shape[1] < Lt:
            keep = torch.empty((B, max(Lt + 64, 2 * (keep.shape[1] if keep is not None else 0))), dtype=torch.int64,
                               device=dev)
            self._ids[cur] = keep
        prev = self._ids[oth] if self._prev_ok else None
        a = self._args
        a.ids, a.B, a.L, a.ld = ids.data_ptr(), B, Lt, Lt
        a.fdf, a.fdf_len = self.fdf.data_ptr(), self.fdf_len
        a.pow_tab, a.pow_len = pow_t.data_ptr(), pow_t.numel()
        if prev is not None:
            a.prev_ids, a.prev_ld, a.prev_B, a.prev_state = prev.data_ptr(), prev.stride(0), prev.shape[0], \
                self._state[oth].data_ptr()
        else:
            a.prev_ids, a.prev_ld, a.prev_B, a.prev_state = None, 0, 0, None
        a.rows, a.mask_lo, a.mask_hi = bufs["rows"].data_ptr(), bufs["mlo"].data_ptr(), bufs["mhi"].data_ptr()
        a.state, a.status = self._state[cur].data_ptr(), self.status.data_ptr()
        a.bits, a.bits_ld = bufs["bits"].data_ptr(), bufs["words"]
        a.dtype = _DTYPE_CODE[dtype]
        a.scores, a.out, a.V, a.ld_scores, a.ld_out = src.data_ptr(), out.data_ptr(), V, src.stride(0), out.stride(0)
        a.unigram_bits = self.core.unigram_bits(V, dev).data_ptr()
        a.eos = int(cfg.eos)
        a.ids_copy, a.copy_ld = keep.data_ptr(), keep.stride(0)
        stream = torch.cuda.current_stream(dev)
        check(lib().fm_processor_shard_prep(self.index._h, ctypes.byref(cfg), ctypes.byref(a),
                                            c_void_p(bufs["facts"].data_ptr()), c_void_p(bufs["rowcase"].data_ptr()),
                                            c_void_p(stream.cuda_stream)), "processor_shard_prep")
        return {"out": out, "B": B, "V": V, "facts": bufs["facts"], "rowcase": bufs["rowcase"], "bits": bufs["bits"],
                "mlo": bufs["mlo"], "mhi": bufs["mhi"], "cfg": cfg, "scores_device": scores.device}

    def finish(self, h, facts_sum, bits_or):
        """The decisions from the summed facts and the epilogue with the ORed
        bits (int32 [B, >= ceil(V/32)]); None when the call needs the host
        path (end markers, boost overflow), which the processor then runs over
        the shards (the same decision on every rank: it depends on the inputs)."""
        from .sharding import HaloExceeded

        a = self._args
        stream = torch.cuda.current_stream(self.dev)
        a.status_host = self.status_h.data_ptr()
        if not self._ev_ready:
            self._ev.record(stream)
            self._ev_ready = True
        a.status_event = self._ev.cuda_event
        check(lib().fm_processor_shard_finish(ctypes.byref(h["cfg"]), ctypes.byref(a),
                                              c_void_p(facts_sum.data_ptr()), c_void_p(h["rowcase"].data_ptr()),
                                              c_void_p(bits_or.data_ptr()), bits_or.stride(0),
                                              c_void_p(stream.cuda_stream)), "processor_shard_finish")
        self._ev.synchronize()
        # the exchange's OR pass ran before this event: a timed-out flag barrier is seen here
        self.sidx.check_exchange()
        st = self._status_np
        if st[0] != 0 or st[1] != st[2]:
            # rows without exactly one end marker / a boost outside the float range: the
            # processor's host path runs next, over the shards (ShardedIndex's sharded forms)
            self._prev_ok = False
            return None
        halo = self.sidx.halo
        if halo is not None and int(st[3]) > halo - 1:
            self._prev_ok = False
            raise HaloExceeded(f"a pattern of {int(st[3])} tokens (force_decoding_from included) needs a halo of "
                               f">= {int(st[3]) + 1}; the shards were built with {halo}")
        self._cur, self._prev_ok = 1 - self._cur, True
        out = h["out"]
        return out if out.device == h["scores_device"] else out.to(h["scores_device"])

    def __call__(self, input_ids, scores, cfg: _PrepConfig, wait: bool = True):
        h = self.prep(input_ids, scores, cfg)
        if h is None:
            return None
        if getattr(self.sidx, "facts_in_payload", False) and self.sidx.group is not None:
            # sparse / peer exchanges: the facts ride in the payload and the OR pass ORs them (> 0 is
            # all k_prep_finish asks of a sum) -- no collective for them; over the peer exchange with
            # the flag barrier the call holds no collective at all
            bits, facts = self.sidx.or_bits(h["mlo"], h["mhi"], h["bits"], h["V"], facts=h["facts"])
            return self.finish(h, facts, bits)
        # the dense exchange (or no group): the peer exchange would pack first so that the facts
        # all_reduce is its barrier
        staged = self.sidx.stage(h["mlo"], h["mhi"], h["bits"], h["V"])
        facts = self.sidx.sum_facts(h["facts"])
        bits = self.sidx.or_bits(h["mlo"], h["mhi"], h["bits"], h["V"], staged=staged)
        return self.finish(h, facts, bits)


class _BatchedCore:
    """Shared machinery: batched ranges, packed allowed bits, fused epilogue."""

    def __init__(self, index):
        self.index = index
        self._uni_cache = {}
        self._prev = {}     # pattern tuple -> (lo, hi) from the previous ranges() call

    # -- index work ---------------------------------------------------------
    def counts(self, patterns: Sequence[Sequence[int]]) -> List[int]:
        if not patterns:
            return []
        sharded = getattr(self.index, "sharded", False)
        if sharded:
            self.index.check_patterns(patterns)
        lo, hi = self.index.get_range_batch(patterns, SHIFT)
        c = (hi.astype(np.int64) - lo.astype(np.int64)).tolist()
        # a doc-sharded index: summed over the ranks (zero exactly when the unsharded count is)
        return self.index.sum_counts(c) if sharded else c

    def ranges(self, patterns: Sequence[Sequence[int]]):
        """get_range of every pattern (index.py:103-114), incrementally: during
        decoding a row's pattern is usually last step's pattern plus one token,
        and get_range is a left-to-right loop of LF steps with an early exit at
        (0, 0), so range(p) == one LF step of range(p[:-1]) by p[-1] -- bit for
        bit the reference's value.  Rows that do not extend a pattern of the
        previous call are searched in full; both kinds go in one launch."""
        if not patterns:
            self._prev = {}
            z = np.zeros(0, dtype=np.uint64)
            return z, z
        if getattr(self.index, "sharded", False):
            self.index.check_patterns(patterns)
        n = self.index.size()
        keys = [tuple(map(int, p)) for p in patterns]
        toks, slo, shi = [], np.zeros(len(keys), dtype=np.uint64), np.zeros(len(keys), dtype=np.uint64)
        for i, k in enumerate(keys):
            prev = self._prev.get(k[:-1]) if k else None
            if prev is not None:
                slo[i], shi[i] = prev
                toks.append(k[-1:])
            else:
                slo[i], shi[i] = 0, n
                toks.append(k)
        lo, hi = self.index.get_range_batch(toks, SHIFT, starts=(slo, shi))
        self._prev = {k: (l, h) for k, l, h in zip(keys, lo.tolist(), hi.tolist())}
        return lo, hi

    def allowed_bits(self, lo: np.ndarray, hi: np.ndarray, vocab: int):
        device = torch.device("cuda", self.index.device)
        lo_t = torch.tensor(lo.astype(np.int64), device=device)
        hi_t = torch.tensor(hi.astype(np.int64), device=device)
        return self.index.allowed_mask(lo_t, hi_t, vocab, SHIFT, packed=True)

    def unigram_bits(self, vocab: int, device):
        key = (device.index if isinstance(device, torch.device) else device, vocab)
        if key not in self._uni_cache:
            words = (vocab + 31) // 32
            bits = np.zeros(words * 32, dtype=np.uint8)
            toks = np.asarray([t for t in self.index.occurring_distinct if 0 <= t < vocab], dtype=np.int64)
            bits[toks] = 1
            packed = np.packbits(bits, bitorder="little").view(np.int32)
            self._uni_cache[key] = torch.from_numpy(packed.copy()).to(device)
        return self._uni_cache[key]

    def epilogue_device(self, scores: torch.Tensor, rows_dev, bits, eos: int) -> torch.Tensor:
        """As ``epilogue`` with the row parameters already on the device."""
        dev_index = torch.device("cuda", self.index.device)
        dtype = scores.dtype
        if dtype not in _DTYPE_CODE:
            raise TypeError(f"unsupported scores dtype {dtype}")
        src = scores.to(dev_index).contiguous()
        out = torch.empty_like(src)
        B, V = src.shape
        uni = self.unigram_bits(V, dev_index)
        stream = torch.cuda.current_stream(dev_index).cuda_stream
        ldb = bits.stride(0) if bits is not None else 0
        check(lib().fm_apply_boosts(_DTYPE_CODE[dtype], c_void_p(src.data_ptr()), c_void_p(out.data_ptr()), B, V,
                                    src.stride(0), out.stride(0),
                                    c_void_p(bits.data_ptr()) if bits is not None else None, ldb,
                                    c_void_p(uni.data_ptr()), c_void_p(rows_dev.data_ptr()), int(eos),
                                    c_void_p(stream)), "apply_boosts")
        return out.to(scores.device)

    def epilogue(self, scores: torch.Tensor, rows: np.ndarray, bits, eos: int) -> torch.Tensor:
        """scores [B, V] (any supported dtype/device) -> scores + mask."""
        dev_index = torch.device("cuda", self.index.device)
        dtype = scores.dtype
        if dtype not in _DTYPE_CODE:
            raise TypeError(f"unsupported scores dtype {dtype}")
        src = scores.to(dev_index).contiguous()
        out = torch.empty_like(src)
        B, V = src.shape
        rp = torch.from_numpy(rows.view(np.uint8).copy()).to(dev_index)
        uni = self.unigram_bits(V, dev_index)
        stream = torch.cuda.current_stream(dev_index).cuda_stream
        ldb = bits.stride(0) if bits is not None else 0
        with torch.cuda.device(dev_index):
            check(lib().fm_apply_boosts(_DTYPE_CODE[dtype], c_void_p(src.data_ptr()), c_void_p(out.data_ptr()), B, V,
                                        src.stride(0), out.stride(0),
                                        c_void_p(bits.data_ptr()) if bits is not None else None, ldb,
                                        c_void_p(uni.data_ptr()), c_void_p(rp.data_ptr()), int(eos),
                                        c_void_p(stream)), "apply_boosts")
        return out.to(scores.device)


def _device_step(core, boost, lrf, fdf):
    """The device path when the index is this engine's GPU index (its
    handle) or a doc-range shard of one (sharding.ShardedIndex), else None
    (e.g. an oracle index in the CPU tests)."""
    from .fm_index import FMIndex as _Engine
    from .sharding import ShardedIndex

    if isinstance(core.index, ShardedIndex):
        return _ShardedDeviceStep(core, boost, lrf, fdf)
    if not isinstance(core.index, _Engine) or not torch.cuda.is_available():
        return None
    return _DeviceStep(core, boost, lrf, fdf)


def _find_marker_rows(input_ids: torch.Tensor, marker: Sequence[int]) -> List[torch.Tensor]:
    """remove_end_marker's result list (…causal_qwen.py:44-56): for every row and
    every occurrence of the marker, the tokens after it (rows without one are
    dropped, rows with several repeat) -- vectorised search, same order."""
    ids = input_ids.cpu()
    m = len(marker)
    out: List[torch.Tensor] = []
    if ids.shape[1] < m:
        return out
    win = ids.unfold(1, m, 1)                                  # [B, L-m+1, m]
    hit = (win == torch.tensor(marker, dtype=ids.dtype)).all(2)
    # slices of the host copy: the callers only read the ids back as lists
    # (one device slice per row would be B tiny device ops per step)
    rr, ii = torch.nonzero(hit, as_tuple=True)
    for r, i in zip(rr.tolist(), ii.tolist()):
        out.append(ids[r, i + m:])
    return out


def _distinct_rule(stop_at_count: int, count: int, last: int, eos: int, pad: int):
    """The per-row distinct-set rule shared by every variant: returns a special
    token, or None for "the allowed set of the row's range"."""
    if stop_at_count > 0 and count <= stop_at_count:
        return eos
    if last == eos:
        return pad
    if last == pad:
        return pad
    return None


class QwenIndexBasedLogitsProcessor:
    """document_constrained_generation_causal_qwen.py:7-214 (soft boosts, think gating)."""

    SYSTEM_TOKENS = [151667, 271, 151668, 271]
    FINISHED_THINKING = (151668, 271)

    def __init__(self, index, num_beams: int, min_new_tokens: int = 5, pad_token_id: int = 0,
                 eos_token_id: int = 2, force_decoding_from: Optional[List[int]] = None, stop_at_count: int = 0,
                 always_allow_eos: bool = False, forced_bos_token_id: Optional[int] = None,
                 length_reward_factor: float = 2.0):
        self.index = index
        self.pad_token_id = pad_token_id
        self.eos_token_id = eos_token_id
        self._num_beams = num_beams
        self.force_decoding_from = force_decoding_from
        self.stop_at_count = stop_at_count
        self.always_allow_eos = always_allow_eos
        self.forced_bos_token_id = forced_bos_token_id
        self.min_new_tokens = min_new_tokens
        self.length_reward_factor = length_reward_factor
        self.BOOST = 10.0
        self.end_marker = [151645, 198, 151644, 77091, 198]
        self._core = _BatchedCore(index)
        self._dev = _device_step(self._core, self.BOOST, length_reward_factor, force_decoding_from)

    @classmethod
    def remove_system_tokens(cls, sent: List[int]) -> List[int]:
        st = cls.SYSTEM_TOKENS
        if len(sent) < len(st):
            return [] if sent == st[: len(sent)] else sent
        return sent[len(st):] if sent[: len(st)] == st else sent

    @classmethod
    def finished_thinking(cls, sent: List[int]) -> bool:
        a, b = cls.FINISHED_THINKING
        return any(sent[i] == a and sent[i + 1] == b for i in range(len(sent) - 1))

    def __call__(self, input_ids, scores):
        return self._process(input_ids, scores)

    def _prep_config(self, dtype) -> _PrepConfig:
        c = _PrepConfig()
        for i, t in enumerate(self.end_marker):
            c.marker[i] = t
        c.marker_len = len(self.end_marker)
        c.think[0], c.think[1] = self.FINISHED_THINKING
        for i, t in enumerate(self.SYSTEM_TOKENS):
            c.sys[i] = t
        c.eos, c.pad = self.eos_token_id, self.pad_token_id
        c.stop_at_count, c.min_new_tokens, c.shift = self.stop_at_count, self.min_new_tokens, SHIFT
        c.num_beams = self._num_beams
        c.flags = PREP_THINK | (PREP_EOS if self.always_allow_eos else 0)
        c.base = 0.0
        c.v_uni_full, c.v_uni_half = _round(self.BOOST, dtype), _round(self.BOOST / 2, dtype)
        return c

    def _process(self, input_ids: torch.LongTensor, scores: torch.FloatTensor) -> torch.Tensor:
        if self._dev is not None:
            out = self._dev(input_ids, scores, _config(self, scores.dtype))
            if out is not None:
                return out
        input_ids = torch.stack(_find_marker_rows(input_ids, self.end_marker))
        B, V = scores.shape
        rows = np.zeros(B, dtype=ROW_DTYPE)
        L = input_ids.size(1)
        if L == 0:
            return self._core.epilogue(scores, rows, None, self.eos_token_id)
        sents = input_ids.view(-1, self._num_beams, L).reshape(-1, L).tolist()
        # think gating + remove_system_tokens + the trailing n-gram rule, whose
        # loop returns on its first iteration: only count([last]) matters
        proc: List[Optional[List[int]]] = []
        need_last = []
        for s in sents:
            if not self.finished_thinking(s):
                proc.append(None)
                continue
            s = self.remove_system_tokens(s)
            proc.append(s)
            if s:
                need_last.append(len(proc) - 1)
        last_counts = self._core.counts([[proc[i][-1]] for i in need_last])
        for i, c in zip(need_last, last_counts):
            if c == 0:
                proc[i] = []
        fdf = self.force_decoding_from
        pat_rows, pats = [], []
        for i, s in enumerate(proc):
            if s and s[-1] not in (self.eos_token_id, self.pad_token_id):
                pat_rows.append(i)
                pats.append((fdf + s) if fdf is not None else s)
        lo, hi = self._core.ranges(pats)
        cnt = {i: int(h) - int(l) for i, l, h in zip(pat_rows, lo.tolist(), hi.tolist())}
        full_lo = np.zeros(B, dtype=np.uint64)
        full_hi = np.zeros(B, dtype=np.uint64)
        for i, l, h in zip(pat_rows, lo.tolist(), hi.tolist()):
            full_lo[i], full_hi[i] = l, h
        bits = self._core.allowed_bits(full_lo, full_hi, V)
        has_bits = bits.ne(0).any(1).cpu().numpy()   # distinct non-empty, one sync for the batch
        dt = scores.dtype
        boost = self.BOOST
        eos_val = None
        if self.always_allow_eos and L >= self.min_new_tokens:
            eos_val = _round(boost * (self.length_reward_factor ** L), dt)
        # per-row fields collected as Python lists and written column-wise
        # (a field store on a numpy record costs ~1 us; B of them per field)
        flags, v_uni, v_dist, special_tok = [0] * B, [0.0] * B, [0.0] * B, [0] * B
        for i, s in enumerate(proc):
            if s is None:
                continue
            if not s:
                f = FLAG_UNIGRAM
                v_uni[i] = _round(boost, dt)
            else:
                special = _distinct_rule(self.stop_at_count, cnt.get(i, 0), s[-1], self.eos_token_id,
                                         self.pad_token_id)
                v_dist[i] = _round(boost * (self.length_reward_factor ** len(s)), dt)
                if special is not None:
                    f = FLAG_SPECIAL | FLAG_UNIGRAM
                    special_tok[i] = special
                    empty = False
                else:
                    f = FLAG_BITS | FLAG_UNIGRAM
                    empty = not bool(has_bits[i])
                v_uni[i] = _round(boost if empty else boost / 2, dt)
            if eos_val is not None:
                f |= FLAG_EOS
            flags[i] = f
        rows["flags"] = flags
        rows["v_uni"] = v_uni
        rows["v_dist"] = v_dist
        rows["special"] = special_tok
        if eos_val is not None:
            rows["v_eos"] = [eos_val if s is not None else 0.0 for s in proc]
        return self._core.epilogue(scores, rows, bits, self.eos_token_id)


class CausalIndexBasedLogitsProcessor:
    """document_constrained_generation_causal.py:7-180 (soft boosts, model-name marker)."""

    END_MARKERS = {"qwen": [151645, 198, 151644, 77091, 198], "llama": [78191, 128007, 271]}

    def __init__(self, index, num_beams: int, model_name: str, pad_token_id: int = 0, eos_token_id: int = 2,
                 force_decoding_from: Optional[List[int]] = None, stop_at_count: int = 0,
                 always_allow_eos: bool = False, forced_bos_token_id: Optional[int] = None,
                 length_reward_factor=2.0):
        self.index = index
        self.pad_token_id = pad_token_id
        self.eos_token_id = eos_token_id
        self._num_beams = num_beams
        self.force_decoding_from = force_decoding_from
        self.stop_at_count = stop_at_count
        self.always_allow_eos = always_allow_eos
        self.forced_bos_token_id = forced_bos_token_id
        self.length_reward_factor = length_reward_factor
        self.BOOST = 10.0
        self.model_name = model_name
        self.end_marker = self.END_MARKERS["llama"]
        if model_name.lower().startswith("qwen"):
            self.end_marker = self.END_MARKERS["qwen"]
        self._core = _BatchedCore(index)
        self._dev = _device_step(self._core, self.BOOST, length_reward_factor, force_decoding_from)

    def __call__(self, input_ids, scores):
        return self._process(input_ids, scores)

    def _prep_config(self, dtype) -> _PrepConfig:
        c = _PrepConfig()
        for i, t in enumerate(self.end_marker):
            c.marker[i] = t
        c.marker_len = len(self.end_marker)
        c.eos, c.pad = self.eos_token_id, self.pad_token_id
        c.stop_at_count, c.shift = self.stop_at_count, SHIFT
        c.num_beams = self._num_beams
        c.flags = PREP_UNI_HALF | ((PREP_EOS | PREP_EOS_ALL) if self.always_allow_eos else 0)
        if self.forced_bos_token_id is not None:
            c.flags |= PREP_SKIP_FIRST
            c.forced_bos = self.forced_bos_token_id
        c.base = 0.0
        c.v_uni_full, c.v_uni_half = _round(self.BOOST, dtype), _round(self.BOOST / 2, dtype)
        c.v_forced = c.v_uni_full
        return c

    def _process(self, input_ids, scores):
        if self._dev is not None:
            # a soft variant: its status (end markers, boost overflow) depends on the
            # input, so the call waits for it (wait=False is for PREP_HARD only)
            out = self._dev(input_ids, scores, _config(self, scores.dtype))
            if out is not None:
                return out
        input_ids = torch.stack(_find_marker_rows(input_ids, self.end_marker))
        B, V = scores.shape
        dt = scores.dtype
        rows = np.zeros(B, dtype=ROW_DTYPE)
        boost = self.BOOST
        if self.forced_bos_token_id is not None:
            if input_ids.size(1) == 0:
                rows["flags"] = FLAG_SPECIAL
                rows["special"] = self.forced_bos_token_id
                rows["v_dist"] = _round(boost, dt)
                return self._core.epilogue(scores, rows, None, self.eos_token_id)
            input_ids = input_ids[:, 1:]
        L = input_ids.size(1)
        bits = None
        if L == 0:
            rows["flags"] = FLAG_UNIGRAM
            rows["v_uni"] = _round(boost, dt)
        else:
            sents = input_ids.view(-1, self._num_beams, L).reshape(-1, L).tolist()
            # trailing n-gram: count([last]) == 0 -> [] (an empty sent returns None ~ [])
            last_counts = self._core.counts([[s[-1]] for s in sents])
            proc = [[] if c == 0 else s for s, c in zip(sents, last_counts)]
            fdf = self.force_decoding_from
            pat_rows, pats = [], []
            for i, s in enumerate(proc):
                if s and s[-1] not in (self.eos_token_id, self.pad_token_id):
                    pat_rows.append(i)
                    pats.append((fdf + s) if fdf is not None else s)
            lo, hi = self._core.ranges(pats)
            cnt = {i: int(h) - int(l) for i, l, h in zip(pat_rows, lo.tolist(), hi.tolist())}
            full_lo = np.zeros(B, dtype=np.uint64)
            full_hi = np.zeros(B, dtype=np.uint64)
            for i, l, h in zip(pat_rows, lo.tolist(), hi.tolist()):
                full_lo[i], full_hi[i] = l, h
            bits = self._core.allowed_bits(full_lo, full_hi, V)
            # column-wise row fields, as in the Qwen variant
            flags, v_uni, v_dist, special_tok = [0] * B, [0.0] * B, [0.0] * B, [0] * B
            for i, s in enumerate(proc):
                if not s:
                    flags[i] = FLAG_UNIGRAM
                    v_uni[i] = _round(boost, dt)
                    continue
                special = _distinct_rule(self.stop_at_count, cnt.get(i, 0), s[-1], self.eos_token_id,
                                         self.pad_token_id)
                v_dist[i] = _round(boost * (self.length_reward_factor ** len(s)), dt)
                v_uni[i] = _round(boost / 2, dt)          # always BOOST / 2 in this variant
                if special is not None:
                    flags[i] = FLAG_SPECIAL | FLAG_UNIGRAM
                    special_tok[i] = special
                else:
                    flags[i] = FLAG_BITS | FLAG_UNIGRAM
            rows["flags"] = flags
            rows["v_uni"] = v_uni
            rows["v_dist"] = v_dist
            rows["special"] = special_tok
        if self.always_allow_eos:
            rows["flags"] |= FLAG_EOS
            rows["v_eos"] = _round(boost * (self.length_reward_factor ** L), dt)
        return self._core.epilogue(scores, rows, bits, self.eos_token_id)


class _HardMaskBase:
    """Shared by the hard-mask (-inf) variants.  With this engine's index a
    call runs on the device (fm_processor_call with FM_PREP_HARD: the pattern
    is every token from ``skip`` on, the range one LF step from the previous
    call's, stop_at_count against the count of the pattern without its last
    token -- which is the previous call's range width); otherwise, and for
    inputs the device path refuses, the batched host path below."""

    SKIP = 0   # leading tokens that are not pattern (seq: the decoder start)

    def _prep_config(self, dtype) -> _PrepConfig:
        c = _PrepConfig()
        c.eos, c.pad = self.eos_token_id, self.pad_token_id
        c.stop_at_count, c.shift = self.stop_at_count, SHIFT
        c.num_beams = self._num_beams
        c.flags = PREP_HARD | ((PREP_EOS | PREP_EOS_ALL) if self.always_allow_eos else 0)
        c.skip = self.SKIP
        if self.forced_bos_token_id is not None:
            c.flags |= PREP_SKIP_FIRST
            c.forced_bos = self.forced_bos_token_id
        c.base = float("-inf")
        c.v_uni_full = c.v_uni_half = c.v_forced = _round(self.BOOST, dtype)
        return c

    def _hard(self, sents: List[List[int]], pattern_of, count_of, V: int, dt, B: int):
        rows = np.zeros(B, dtype=ROW_DTYPE)
        rows["base"] = float("-inf")
        boost = _round(self.BOOST, dt)
        fdf = self.force_decoding_from if self.force_decoding_from is not None else []
        pats, cpats, pat_rows = [], [], []
        for i, s in enumerate(sents):
            if s[-1] in (self.eos_token_id, self.pad_token_id):
                continue
            pat_rows.append(i)
            pats.append(fdf + pattern_of(s))
            cpats.append(fdf + count_of(s))
        lo, hi = self._core.ranges(pats)
        counts = self._core.counts(cpats)
        cnt = dict(zip(pat_rows, counts))
        full_lo = np.zeros(B, dtype=np.uint64)
        full_hi = np.zeros(B, dtype=np.uint64)
        for i, l, h in zip(pat_rows, lo.tolist(), hi.tolist()):
            full_lo[i], full_hi[i] = l, h
        bits = self._core.allowed_bits(full_lo, full_hi, V)
        for i, s in enumerate(sents):
            r = rows[i]
            special = _distinct_rule(self.stop_at_count, cnt.get(i, 0), s[-1], self.eos_token_id,
                                     self.pad_token_id)
            r["v_dist"] = boost
            if special is not None:
                r["flags"] = FLAG_SPECIAL
                r["special"] = special
            else:
                r["flags"] = FLAG_BITS
        return rows, bits


class VllmIndexBasedLogitsProcessor(_HardMaskBase):
    """document_constrained_generation_vllm.py:6-137 (vLLM V0 per-sequence hard mask)."""

    def __init__(self, index, num_beams: int, pad_token_id: int = 0, eos_token_id: int = 2,
                 force_decoding_from: Optional[List[int]] = None, stop_at_count: int = 0,
                 always_allow_eos: bool = False, forced_bos_token_id: Optional[int] = None):
        self.index = index
        self.pad_token_id = pad_token_id
        self.eos_token_id = eos_token_id
        self._num_beams = num_beams
        self.force_decoding_from = force_decoding_from
        self.stop_at_count = stop_at_count
        self.always_allow_eos = always_allow_eos
        self.forced_bos_token_id = forced_bos_token_id
        self.BOOST = 0.0
        self._core = _BatchedCore(index)
        self._dev = _device_step(self._core, self.BOOST, 1.0, force_decoding_from)
        self._ids_dev = None        # the sequence's ids on the device (see _device_ids)
        self._ids_pin = None
        self._ids_prev = ()
        self._ids_ev = None         # recorded behind the last staged copy

    def clone(self):
        return VllmIndexBasedLogitsProcessor(num_beams=self._num_beams, index=self.index,
                                             pad_token_id=self.pad_token_id, eos_token_id=self.eos_token_id,
                                             force_decoding_from=self.force_decoding_from,
                                             stop_at_count=self.stop_at_count,
                                             always_allow_eos=self.always_allow_eos,
                                             forced_bos_token_id=self.forced_bos_token_id)

    def _device_ids(self, toks):
        """The sequence's output ids as a device int64 [1, L] view.  vLLM hands
        each sequence's clone its whole output tuple every step, one token
        longer than last time: only the tokens beyond the part already on the
        device are staged (pinned) and copied -- one 8-byte copy per step
        instead of the whole tuple (the prefix is compared on the host first, so
        a tuple that does not extend the previous one is uploaded whole)."""
        L = len(toks)
        buf = self._ids_dev
        if buf is None or buf.shape[1] < max(L, 1):
            cap = max(64, 2 * L)
            self._ids_dev = buf = torch.empty((1, cap), dtype=torch.int64, device=self._dev.dev)
            self._ids_pin = torch.empty(cap, dtype=torch.int64).pin_memory()
            self._ids_pin_np = self._ids_pin.numpy()
            self._ids_prev = ()
            self._ids_ev = None
        prev = self._ids_prev
        k = len(prev) if len(prev) <= L and toks[:len(prev)] == prev else 0
        if L > k:
            if k < len(prev) and self._ids_ev is not None:
                self._ids_ev.synchronize()      # staged slots about to be rewritten: their last copy must be done
            self._ids_pin_np[k:L] = toks[k:L]
            buf[0, k:L].copy_(self._ids_pin[k:L], non_blocking=True)
            if self._ids_ev is None:
                self._ids_ev = torch.cuda.Event()
            self._ids_ev.record(torch.cuda.current_stream(buf.device))
        self._ids_prev = toks
        return buf[:, :L]

    def __call__(self, input_ids, scores):
        scores = scores.unsqueeze(0)
        if self._dev is not None:
            out = self._dev(self._device_ids(tuple(input_ids)), scores, _config(self, scores.dtype), wait=False)
            if out is not None:
                return out
        input_ids = torch.tensor([list(input_ids)], dtype=torch.long)
        B, V = scores.shape
        dt = scores.dtype
        boost = _round(self.BOOST, dt)
        if self.forced_bos_token_id is not None:
            if input_ids.size(1) == 0:
                rows = np.zeros(B, dtype=ROW_DTYPE)
                rows["base"] = float("-inf")
                rows["flags"] = FLAG_SPECIAL
                rows["special"] = self.forced_bos_token_id
                rows["v_dist"] = boost
                return self._core.epilogue(scores, rows, None, self.eos_token_id)
            input_ids = input_ids[:, 1:]
        L = input_ids.size(1)
        bits = None
        if L == 0:
            rows = np.zeros(B, dtype=ROW_DTYPE)
            rows["base"] = float("-inf")
            rows["flags"] = FLAG_UNIGRAM
            rows["v_uni"] = boost
        else:
            sents = input_ids.view(-1, self._num_beams, L).reshape(-1, L).tolist()
            rows, bits = self._hard(sents, lambda s: s, lambda s: s[:-1], V, dt, B)
        if self.always_allow_eos:
            rows["flags"] |= FLAG_EOS
            rows["v_eos"] = boost
        return self._core.epilogue(scores, rows, bits, self.eos_token_id)


class SeqIndexBasedLogitsProcessor(_HardMaskBase):
    """document_constrained_generation_seq.py:6-123 (seq2seq hard mask; decoder start skipped)."""

    SKIP = 1

    def __init__(self, index, num_beams: int, pad_token_id: int = 0, eos_token_id: int = 2,
                 force_decoding_from: Optional[List[int]] = None, stop_at_count: int = 0,
                 always_allow_eos: bool = False, forced_bos_token_id: Optional[int] = None):
        self.index = index
        self.pad_token_id = pad_token_id
        self.eos_token_id = eos_token_id
        self._num_beams = num_beams
        self.force_decoding_from = force_decoding_from
        self.stop_at_count = stop_at_count
        self.always_allow_eos = always_allow_eos
        self.forced_bos_token_id = forced_bos_token_id
        self.BOOST = 0.0
        self._core = _BatchedCore(index)
        self._dev = _device_step(self._core, self.BOOST, 1.0, force_decoding_from)

    def __call__(self, input_ids, scores):
        return self._process(input_ids, scores)

    def _process(self, input_ids, scores):
        if self._dev is not None:
            out = self._dev(input_ids, scores, _config(self, scores.dtype), wait=False)
            if out is not None:
                return out
        B, V = scores.shape
        dt = scores.dtype
        boost = _round(self.BOOST, dt)
        if self.forced_bos_token_id is not None:
            if input_ids.size(1) == 1:
                rows = np.zeros(B, dtype=ROW_DTYPE)
                rows["base"] = float("-inf")
                rows["flags"] = FLAG_SPECIAL
                rows["special"] = self.forced_bos_token_id
                rows["v_dist"] = boost
                return self._core.epilogue(scores, rows, None, self.eos_token_id)
            input_ids = input_ids[:, 1:]
        L = input_ids.size(1)
        bits = None
        if L == 1:
            rows = np.zeros(B, dtype=ROW_DTYPE)
            rows["base"] = float("-inf")
            rows["flags"] = FLAG_UNIGRAM
            rows["v_uni"] = boost
        else:
            sents = input_ids.view(-1, self._num_beams, L).reshape(-1, L).tolist()
            rows, bits = self._hard(sents, lambda s: s[1:], lambda s: s[1:-1], V, dt, B)
        if self.always_allow_eos:
            rows["flags"] |= FLAG_EOS
            rows["v_eos"] = boost
        return self._core.epilogue(scores, rows, bits, self.eos_token_id)


# reference class name of the primary processor
IndexBasedLogitsProcessor = QwenIndexBasedLogitsProcessor

__all__ = ["QwenIndexBasedLogitsProcessor", "CausalIndexBasedLogitsProcessor", "SeqIndexBasedLogitsProcessor",
           "VllmIndexBasedLogitsProcessor", "IndexBasedLogitsProcessor"]
