"""``FMIndex`` -- the SWIG surface of ``cpp_modules.fm_index`` on the MI355X engine.

Reference: ``cpp_modules_linux/fm_index.hpp:20-45`` / ``fm_index.cpp:27-209``
(SWIG module ``fm_index.i``).  Same method names, argument meaning, return
shapes (tuples, as SWIG returns for ``std::vector``) and error behaviour
(``OverflowError`` for negative / oversize unsigned arguments, ``TypeError``
for non-integers).  Every query runs on the GPU holding the index; the
batched ``*_batch`` / ``allowed_mask`` / ``decode_step`` methods take torch
tensors resident on that GPU and are stream-ordered on torch's current stream.
"""
from __future__ import annotations

import ctypes
import itertools
import os
from ctypes import byref, c_uint32, c_uint64, c_void_p
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

from ._lib import FMIndexError, check, lib

U64_MAX = (1 << 64) - 1


def _u64(v, method: str, argno: int, typ: str = "size_type") -> int:
    if isinstance(v, (bool,)) or not isinstance(v, (int, np.integer)):
        raise TypeError(f"in method 'FMIndex_{method}', argument {argno} of type '{typ}'")
    v = int(v)
    if v < 0 or v > U64_MAX:
        raise OverflowError(f"in method 'FMIndex_{method}', argument {argno} of type '{typ}'")
    return v


def _u64_vec(values, method: str, argno: int) -> np.ndarray:
    if isinstance(values, np.ndarray):
        arr = values
    else:
        values = list(values)
        for v in values:
            if isinstance(v, bool) or not isinstance(v, (int, np.integer)):
                raise TypeError(f"in method 'FMIndex_{method}', argument {argno} of type "
                                "'std::vector< unsigned long,std::allocator< unsigned long > >'")
        arr = np.asarray(values, dtype=object) if values else np.zeros(0, dtype=np.int64)
    if arr.size:
        mn = int(arr.min())
        mx = int(arr.max())
        if mn < 0 or mx > U64_MAX:
            raise OverflowError(f"in method 'FMIndex_{method}', argument {argno} of type "
                                "'std::vector< unsigned long,std::allocator< unsigned long > >'")
    return np.ascontiguousarray(arr.astype(np.uint64))


def _ptr(a: np.ndarray, ctype=c_uint64):
    return a.ctypes.data_as(ctypes.POINTER(ctype))


def _default_device() -> int:
    env = os.environ.get("FMIDX_DEVICE")
    if env is not None:
        return int(env)
    try:
        import torch

        if torch.cuda.is_available():
            return int(torch.cuda.current_device())
    except Exception:  # pragma: no cover - torch is optional for the SWIG surface
        pass
    return 0


def payload_capacity(B: int, vocab: int) -> int:
    """uint32 words a sparse-exchange payload of B rows may need (fm_shard_payload_capacity)."""
    out = c_uint64()
    check(lib().fm_shard_payload_capacity(int(B), int(vocab), ctypes.byref(out)), "shard_payload_capacity")
    return int(out.value)


def _stream_of(t) -> int:
    """The raw handle of the current stream on t's device: torch's C-level
    getter (~0.1 us) where it exists -- torch.cuda.current_stream() builds a
    Stream object on every call (~2 us, a quarter of a decode-step launch's
    host cost, tools/probe_launch_host.py)."""
    import torch

    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    raw = getattr(torch._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return int(raw(idx))
    return int(torch.cuda.current_stream(t.device).cuda_stream)


class FMIndex:
    """Drop-in for the SWIG proxy class ``cpp_modules.fm_index.FMIndex``."""

    def __init__(self, device: Optional[int] = None, options=None):
        """``options``: the index structures this handle builds
        (fmidx.options: a BuildOptions, a profile name -- "default" /
        "compact" -- or a dict of fm_build_options fields; None = default)."""
        from .options import as_build_options

        self._h = c_void_p()
        self._device = _default_device() if device is None else int(device)
        check(lib().fm_create(byref(self._h), self._device), "FMIndex()")
        o = as_build_options(options)
        if o is not None:
            check(lib().fm_set_build_options(self._h, byref(o)), "set_build_options")

    def build_options(self) -> dict:
        """The fm_build_options in force on this handle (FMIDX_BUILD_OPTIONS applied)."""
        from .options import BuildOptions

        o = BuildOptions()
        check(lib().fm_get_build_options(self._h, byref(o)), "get_build_options")
        return o.as_dict()

    # -- lifecycle ----------------------------------------------------------
    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().fm_destroy(h)
            except Exception:
                pass
            self._h = c_void_p()

    @property
    def device(self) -> int:
        return self._device

    # -- construction (fm_index.cpp:33-48) ----------------------------------
    def initialize(self, data) -> None:
        arr = _u64_vec(data, "initialize", 2)
        check(lib().fm_initialize(self._h, _ptr(arr), arr.size), "initialize")

    def initialize_from_file(self, file: str, width: int) -> None:
        if not isinstance(file, str):
            raise TypeError("in method 'FMIndex_initialize_from_file', argument 2 of type 'std::string const'")
        check(lib().fm_initialize_from_file(self._h, file.encode(), int(width)), "initialize_from_file")

    def initialize_from_bwt_device(self, bwt, sa=None, text=None) -> None:
        """Device build from a uint32/int32 BWT tensor already in HBM."""
        import torch

        assert bwt.is_cuda and bwt.dtype in (torch.int32,) and bwt.is_contiguous()
        stream = _stream_of(bwt)
        check(lib().fm_initialize_from_bwt_device(
            self._h, c_void_p(bwt.data_ptr()), bwt.numel(),
            c_void_p(sa.data_ptr()) if sa is not None else None,
            c_void_p(text.data_ptr()) if text is not None else None,
            c_void_p(stream)), "initialize_from_bwt_device")

    def initialize_from_text_device(self, text, keep_sa_text: bool = False) -> None:
        """GPU construction (suffix sort + BWT + index) from T' (int32 tensor in
        HBM, ending with the unique sentinel 0); replaces sdsl construct_im
        (fm_index.cpp:33-41) for corpora too large for host suffix sorting."""
        import torch

        assert text.is_cuda and text.dtype == torch.int32 and text.is_contiguous()
        check(lib().fm_initialize_from_text_device(self._h, c_void_p(text.data_ptr()), text.numel(),
                                                   1 if keep_sa_text else 0, c_void_p(_stream_of(text))),
              "initialize_from_text_device")

    # -- SWIG surface --------------------------------------------------------
    def size(self) -> int:
        out = c_uint64()
        check(lib().fm_size(self._h, byref(out)), "size")
        return int(out.value)

    def sigma(self) -> int:
        out = c_uint64()
        check(lib().fm_sigma(self._h, byref(out)), "sigma")
        return int(out.value)

    def backward_search_step(self, symbol, low, high) -> Tuple[int, int]:
        """fm_index.cpp:67-97."""
        s = _u64(symbol, "backward_search_step", 2, "char_type")
        lo = _u64(low, "backward_search_step", 3)
        hi = _u64(high, "backward_search_step", 4)
        out = (c_uint64 * 2)()
        check(lib().fm_backward_search_step(self._h, s, lo, hi, out), "backward_search_step")
        return (int(out[0]), int(out[1]))

    def backward_search_multi(self, query) -> Tuple[int, int]:
        """fm_index.cpp:55-65."""
        q = _u64_vec(query, "backward_search_multi", 2)
        out = (c_uint64 * 2)()
        check(lib().fm_backward_search_multi(self._h, _ptr(q), q.size, out), "backward_search_multi")
        return (int(out[0]), int(out[1]))

    def _width(self, low: int, high: int) -> int:
        n = self.size()
        if low == high:
            return 0
        high = min(high, n)
        return max(0, high - low)

    def distinct(self, low, high) -> Tuple[int, ...]:
        """fm_index.cpp:99-117."""
        lo = _u64(low, "distinct", 2)
        hi = _u64(high, "distinct", 3)
        cap = max(1, min(self._width(lo, hi), self.sigma()))
        buf = np.zeros(cap, dtype=np.uint64)
        k = c_uint64()
        check(lib().fm_distinct(self._h, lo, hi, _ptr(buf), cap, byref(k)), "distinct")
        return tuple(int(x) for x in buf[: k.value])

    def distinct_count(self, low, high) -> Tuple[int, ...]:
        """fm_index.cpp:119-144: interleaved (symbol, count), ascending."""
        lo = _u64(low, "distinct_count", 2)
        hi = _u64(high, "distinct_count", 3)
        cap = 2 * max(1, min(self._width(lo, hi), self.sigma()))
        buf = np.zeros(cap, dtype=np.uint64)
        k = c_uint64()
        check(lib().fm_distinct_count(self._h, lo, hi, _ptr(buf), cap, byref(k)), "distinct_count")
        return tuple(int(x) for x in buf[: 2 * k.value])

    def _distinct_count_multi_arrays(self, lows: np.ndarray, highs: np.ndarray):
        m = lows.size
        n = self.size()
        sigma = self.sigma()
        hc = np.minimum(highs, np.uint64(n))
        width = np.where((lows == highs) | (lows >= hc), 0, hc - lows)
        cap = int(2 * np.minimum(width, np.uint64(sigma)).astype(np.uint64).sum())
        out = np.zeros(max(1, cap), dtype=np.uint64)
        offs = np.zeros(m + 1, dtype=np.uint64)
        check(lib().fm_distinct_count_multi(self._h, _ptr(lows), _ptr(highs), m, _ptr(out),
                                            max(1, cap), _ptr(offs)), "distinct_count_multi")
        return out, offs

    def distinct_count_multi(self, lows, highs):
        """fm_index.cpp:146-166: one batched GPU launch for all ranges."""
        lo = _u64_vec(lows, "distinct_count_multi", 2)
        hi = _u64_vec(highs, "distinct_count_multi", 3)
        if lo.size != hi.size:
            raise ValueError("lows and highs differ in length")
        out, offs = self._distinct_count_multi_arrays(lo, hi)
        flat = out.tolist()
        o = offs.tolist()
        return tuple(tuple(flat[2 * o[i]: 2 * o[i + 1]]) for i in range(lo.size))

    def locate(self, row) -> int:
        """fm_index.cpp:168-172."""
        r = _u64(row, "locate", 2)
        out = c_uint64()
        check(lib().fm_locate(self._h, r, byref(out)), "locate")
        return int(out.value)

    def extract_text(self, begin, end) -> Tuple[int, ...]:
        """fm_index.cpp:174-194."""
        b = _u64(begin, "extract_text", 2)
        e = _u64(end, "extract_text", 3)
        if e <= b:
            return tuple()
        n = self.size()
        cap = max(1, min(e, n) - b) if min(e, n) > b else 1
        buf = np.zeros(cap, dtype=np.uint64)
        ln = c_uint64()
        check(lib().fm_extract_text(self._h, b, e, _ptr(buf), cap, byref(ln)), "extract_text")
        return tuple(int(x) for x in buf[: ln.value])

    def save(self, path: str) -> None:
        check(lib().fm_save(self._h, str(path).encode()), "save")

    # -- engine extensions ---------------------------------------------------
    def stats(self) -> dict:
        vals = [c_uint64() for _ in range(5)]
        check(lib().fm_stats(self._h, *[byref(v) for v in vals]), "stats")
        keys = ["levels", "wm_bytes", "bwt_bytes", "bitmap_bytes", "bitmap_block"]
        out = {k: int(v.value) for k, v in zip(keys, vals)}
        out["follow_bytes"] = int(self.build_options()["follow_bitmaps"] != 0 and out["bitmap_block"] > 0)
        ex = [c_uint64() for _ in range(5)]
        check(lib().fm_stats_ex(self._h, *[byref(v) for v in ex]), "stats_ex")
        for k, v in zip(["lf_levels", "lf_wm_bytes", "cache_nodes", "cache_bytes", "cache_min"], ex):
            out[k] = int(v.value)
        tr = [c_uint64() for _ in range(3)]
        check(lib().fm_stats_trans(self._h, *[byref(v) for v in tr]), "stats_trans")
        for k, v in zip(["trans_entries", "trans_dropped", "trans_bytes"], tr):
            out[k] = int(v.value)
        tc = c_uint32()
        check(lib().fm_stats_trans_complete(self._h, byref(tc)), "stats_trans_complete")
        out["trans_complete"] = int(tc.value)
        mem = [c_uint64() for _ in range(3)]
        check(lib().fm_stats_mem(self._h, *[byref(v) for v in mem]), "stats_mem")
        for k, v in zip(["lf_e_bytes", "sample_bytes", "device_bytes"], mem):
            out[k] = int(v.value)
        bv = c_uint64()
        check(lib().fm_stats_views(self._h, byref(bv)), "stats_views")
        out["bwt_view_bytes"] = int(bv.value)     # a materialised BWT copy (device_bwt), outside device_bytes
        return out

    def cache_contains(self, lo, hi):
        """uint8 device tensor: 1 where [lo, hi) has a cached range bitmap."""
        import torch

        out = torch.empty(lo.numel(), dtype=torch.uint8, device=lo.device)
        check(lib().fm_cache_lookup_batch(self._h, c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()), lo.numel(),
                                          c_void_p(out.data_ptr()), c_void_p(_stream_of(lo))), "cache_lookup_batch")
        return out

    def get_range_batch(self, patterns: Sequence[Sequence[int]], shift: int = 0,
                        starts: Optional[Tuple[Sequence[int], Sequence[int]]] = None):
        """get_range (index.py:103-114) for many patterns in one GPU launch.
        Returns (lows, highs) as uint64 numpy arrays."""
        m = len(patterns)
        lens = np.fromiter(map(len, patterns), dtype=np.int64, count=m)
        offs = np.zeros(m + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        # (chain + fromiter: ~2.7x faster than a per-token int() generator; this
        # packing is most of the call's host time at B = 256)
        toks = np.fromiter(itertools.chain.from_iterable(patterns), dtype=np.int64, count=int(offs[-1]))
        lo_out = np.zeros(max(1, m), dtype=np.uint64)
        hi_out = np.zeros(max(1, m), dtype=np.uint64)
        if m == 0:
            return lo_out[:0], hi_out[:0]
        li = hi_in = None
        if starts is not None:
            li = np.ascontiguousarray(np.asarray(starts[0], dtype=np.uint64))
            hi_in = np.ascontiguousarray(np.asarray(starts[1], dtype=np.uint64))
        check(lib().fm_get_range_batch(
            self._h, _ptr(toks, ctypes.c_int64), _ptr(offs, ctypes.c_int64), m, int(shift),
            _ptr(li) if li is not None else None, _ptr(hi_in) if hi_in is not None else None,
            _ptr(lo_out), _ptr(hi_out)), "get_range_batch")
        return lo_out, hi_out

    # torch-tensor batched hot path (device pointers, current stream)
    def lf_step_batch(self, tokens, lo, hi, shift: int, lo_out=None, hi_out=None,
                      reset_below: int = -(1 << 63)):
        lo_out = lo if lo_out is None else lo_out
        hi_out = hi if hi_out is None else hi_out
        check(lib().fm_lf_step_batch(self._h, c_void_p(tokens.data_ptr()), int(shift), int(reset_below),
                                     c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()),
                                     c_void_p(lo_out.data_ptr()), c_void_p(hi_out.data_ptr()),
                                     lo.numel(), c_void_p(_stream_of(lo))), "lf_step_batch")
        return lo_out, hi_out

    def backward_search_batch(self, tokens, offsets, shift: int, lo_out, hi_out, lo_in=None, hi_in=None):
        check(lib().fm_backward_search_batch(
            self._h, c_void_p(tokens.data_ptr()), c_void_p(offsets.data_ptr()), lo_out.numel(), int(shift),
            c_void_p(lo_in.data_ptr()) if lo_in is not None else None,
            c_void_p(hi_in.data_ptr()) if hi_in is not None else None,
            c_void_p(lo_out.data_ptr()), c_void_p(hi_out.data_ptr()),
            c_void_p(_stream_of(lo_out))), "backward_search_batch")
        return lo_out, hi_out

    def allowed_mask(self, lo, hi, vocab: int, shift: int, out=None, packed: bool = False):
        """bool/uint8 [m, vocab] (or int32 [m, ceil(vocab/32)] when packed)."""
        import torch

        m = lo.numel()
        if out is None:
            if packed:
                out = torch.empty((m, (vocab + 31) // 32), dtype=torch.int32, device=lo.device)
            else:
                out = torch.empty((m, vocab), dtype=torch.uint8, device=lo.device)
        ld = out.stride(0) * out.element_size()
        check(lib().fm_allowed_mask_batch(self._h, c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()), m,
                                          c_void_p(out.data_ptr()), ld, int(vocab), int(shift),
                                          1 if packed else 0, c_void_p(_stream_of(lo))), "allowed_mask")
        return out

    def decode_step(self, tokens, lo, hi, mask, vocab: int, shift: int, reset_below: int = -(1 << 63),
                    packed: bool = False, lo_out=None, hi_out=None):
        """Fused LF step + allowed mask (one launch).  With ``lo_out``/``hi_out``
        the new state goes there (must not alias lo/hi); otherwise lo/hi are
        updated in place through a temporary."""
        import torch

        inplace = lo_out is None
        if inplace and vocab:
            lo_out = torch.empty_like(lo)
            hi_out = torch.empty_like(hi)
        elif inplace:
            lo_out, hi_out = lo, hi
        ld = mask.stride(0) * mask.element_size()
        check(lib().fm_decode_step_batch(self._h, c_void_p(tokens.data_ptr()), int(shift), int(reset_below),
                                         c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()),
                                         c_void_p(lo_out.data_ptr()), c_void_p(hi_out.data_ptr()), lo.numel(),
                                         c_void_p(mask.data_ptr()), ld, int(vocab), 1 if packed else 0,
                                         c_void_p(_stream_of(lo))), "decode_step")
        if inplace and vocab:
            lo.copy_(lo_out)
            hi.copy_(hi_out)
        return mask

    def decode_step_payload(self, tokens, lo, hi, lo_out, hi_out, payload, vocab: int, shift: int,
                            reset_below: int = -(1 << 63), payload_alt=None, step=None):
        """The fused LF step writing the shard exchange's payload with fixed row
        slots (fm_decode_step_payload): per row the BWT slice of its new range
        when narrower than ceil(vocab/32) words and streamed whole, else its
        packed bitmap -- what PeerExchange's readers take in place, no pack
        pass.  ``payload``: int32, >= payload_capacity(B, vocab) words.  The
        state may be updated in place (lo_out is lo).  ``step`` (the flag
        barrier's device counter, int32 [1]) with ``payload_alt``: the kernel
        writes ``payload`` on an even counter and ``payload_alt`` on an odd one."""
        if (step is None) != (payload_alt is None):
            raise ValueError("decode_step_payload: payload_alt and step go together")
        if payload_alt is not None and payload_alt.numel() < payload.numel():
            raise ValueError("decode_step_payload: payload_alt smaller than payload")
        check(lib().fm_decode_step_payload(self._h, c_void_p(tokens.data_ptr()), int(shift), int(reset_below),
                                           c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()),
                                           c_void_p(lo_out.data_ptr()), c_void_p(hi_out.data_ptr()), lo.numel(),
                                           c_void_p(payload.data_ptr()), payload.numel(), int(vocab),
                                           c_void_p(payload_alt.data_ptr()) if payload_alt is not None else None,
                                           c_void_p(step.data_ptr()) if step is not None else None,
                                           c_void_p(_stream_of(lo))), "decode_step_payload")
        return payload

    def decode_step_payload_signal(self, tokens, lo, hi, payload, payload_alt, step, flag_ptrs, world: int, done,
                                   vocab: int, shift: int, reset_below: int = -(1 << 63)):
        """decode_step_payload in place with the flag barrier's signal fused in
        (fm_decode_step_payload_signal): the last workgroup posts the step to the
        ``world`` flag words at ``flag_ptrs`` (int64 device addresses) and
        advances ``step``; ``done`` (int32 [288], zero: nine counters on their own
        128-B lines) counts the workgroups."""
        if done.numel() < 9 * 32:
            raise ValueError("decode_step_payload_signal: done needs 9 * 32 int32 words")
        check(lib().fm_decode_step_payload_signal(
            self._h, c_void_p(tokens.data_ptr()), int(shift), int(reset_below), c_void_p(lo.data_ptr()),
            c_void_p(hi.data_ptr()), c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()), lo.numel(),
            c_void_p(payload.data_ptr()), payload.numel(), int(vocab), c_void_p(payload_alt.data_ptr()),
            c_void_p(step.data_ptr()), c_void_p(flag_ptrs.data_ptr()), int(world), c_void_p(done.data_ptr()),
            c_void_p(_stream_of(lo))), "decode_step_payload_signal")
        return payload

    def shard_pack(self, lo, hi, bits, vocab: int, payload=None, facts=None):
        """The sparse exchange payload of this shard's rows (fm_shard_pack):
        per row its BWT slice when narrower than a bitmap, else its packed
        allowed-bit row from ``bits`` (int32 [B, >= ceil(vocab/32)], the
        decode step's packed output).  ``facts`` (int32 [3, B], a processor
        call's per-row facts): stored in the payload's facts area
        (fm_shard_pack_facts), for the OR pass to OR.  Returns the int32
        payload tensor (capacity for the worst case; word 0 = words used)."""
        import torch

        B = lo.numel()
        if payload is None or payload.numel() < payload_capacity(B, vocab):   # the batch may have grown
            payload = torch.empty(payload_capacity(B, vocab), dtype=torch.int32, device=lo.device)
        if facts is not None:
            if not (facts.dtype == torch.int32 and facts.is_contiguous() and facts.numel() == 3 * B):
                raise ValueError(f"shard_pack: facts must be a contiguous int32 [3, {B}] tensor")
            check(lib().fm_shard_pack_facts(self._h, c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()), B,
                                            c_void_p(bits.data_ptr()), bits.stride(0), int(vocab),
                                            c_void_p(facts.data_ptr()), c_void_p(payload.data_ptr()),
                                            payload.numel(), c_void_p(_stream_of(lo))), "shard_pack_facts")
            return payload
        check(lib().fm_shard_pack(self._h, c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()), B,
                                  c_void_p(bits.data_ptr()), bits.stride(0), int(vocab), c_void_p(payload.data_ptr()),
                                  payload.numel(), c_void_p(_stream_of(lo))), "shard_pack")
        return payload

    def distinct_count_batch(self, lo, hi, cap=None):
        """Device interval_symbols for m ranges -> (syms, counts, k, cap_off).
        ``cap`` (int64 device tensor [m]) overrides the per-row capacity
        (default min(width, sigma), always enough); a row with more distinct
        symbols than its capacity reports k = UINT64_MAX (-1 here) and writes
        nothing."""
        import torch

        n = self.size()
        sigma = self.sigma()
        if cap is None:
            hc = torch.clamp(hi, max=n)
            width = torch.where((lo == hi) | (lo >= hc), torch.zeros_like(lo), hc - lo)
            cap = torch.clamp(width, max=sigma)
        cap_off = torch.zeros(lo.numel() + 1, dtype=torch.int64, device=lo.device)
        torch.cumsum(cap, 0, out=cap_off[1:])
        total = int(cap_off[-1].item())
        syms = torch.empty(max(1, total), dtype=torch.int64, device=lo.device)
        counts = torch.empty(max(1, total), dtype=torch.int64, device=lo.device)
        k = torch.empty(lo.numel(), dtype=torch.int64, device=lo.device)
        check(lib().fm_distinct_count_batch(self._h, c_void_p(lo.data_ptr()), c_void_p(hi.data_ptr()),
                                            lo.numel(), c_void_p(cap_off.data_ptr()), total,
                                            c_void_p(syms.data_ptr()), c_void_p(counts.data_ptr()),
                                            c_void_p(k.data_ptr()), c_void_p(_stream_of(lo))),
              "distinct_count_batch")
        return syms, counts, k, cap_off

    def locate_batch(self, rows):
        """SA[row] for an int64 device tensor of rows (fm_index.cpp:168-172 for
        all rows at once; UINT64_MAX -- as int64, -1 -- for rows >= size())."""
        import torch

        out = torch.empty(rows.numel(), dtype=torch.int64, device=rows.device)
        check(lib().fm_locate_batch(self._h, c_void_p(rows.data_ptr()), rows.numel(), c_void_p(out.data_ptr()),
                                    c_void_p(_stream_of(rows))), "locate_batch")
        return out

    def extract_batch(self, begins: Sequence[int], ends: Sequence[int]) -> List[Tuple[int, ...]]:
        """extract_text (fm_index.cpp:174-194) of many (begin, end) pairs in one
        launch; same results and clamping as ``extract_text`` (an empty tuple
        when end <= begin)."""
        import torch

        n = self.size()
        m = len(begins)
        if m != len(ends):
            raise ValueError("begins and ends differ in length")
        b = [_u64(x, "extract_text", 2) for x in begins]
        e = [_u64(x, "extract_text", 3) for x in ends]
        lens = []
        for x, y in zip(b, e):
            if y <= x:
                lens.append(0)
                continue
            if min(y, n) <= x:
                raise FMIndexError(f"extract_text: begin {x} >= clamped end {min(y, n)} (unbounded in the reference)")
            lens.append(min(y, n) - x)
        if m == 0:
            return []
        dev = torch.device("cuda", self._device)
        off = torch.tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), device=dev)
        bt = torch.tensor(np.asarray(b, dtype=np.uint64).view(np.int64), device=dev)
        et = torch.tensor(np.asarray(e, dtype=np.uint64).view(np.int64), device=dev)
        out = torch.empty(max(1, int(off[-1])), dtype=torch.int64, device=dev)
        check(lib().fm_extract_batch(self._h, c_void_p(bt.data_ptr()), c_void_p(et.data_ptr()), c_void_p(off.data_ptr()),
                                     m, c_void_p(out.data_ptr()), c_void_p(_stream_of(bt))), "extract_batch")
        flat = out.cpu().tolist()
        o = off.cpu().tolist()
        return [tuple(flat[o[i]:o[i + 1]]) for i in range(m)]

    def device_bwt(self):
        """The handle's BWT (uint32[n] in HBM) as an int32 torch tensor on
        the index's device (read-only by contract) -- for samplers, traces and
        the CPU baseline.  With the plain BWT freed (the default: E holds the
        symbols) this MATERIALISES an n * 4-byte copy held by the handle
        (stats()["bwt_view_bytes"]); release_bwt_view() frees it, after which
        the tensor must not be used."""
        import torch

        idx = self

        class _View:
            __cuda_array_interface__ = {"shape": (self.size(),), "typestr": "<i4",
                                        "data": (self.device_bwt_ptr(), False), "version": 2, "strides": None}

            def __init__(self):
                self.owner = idx

        with torch.cuda.device(self._device):
            t = torch.as_tensor(_View(), device=torch.device("cuda", self._device))
        return t

    def release_bwt_view(self) -> None:
        """Free the BWT copy device_bwt() materialised (synchronises the
        device; tensors from device_bwt() are dead afterwards)."""
        check(lib().fm_release_bwt_view(self._h), "release_bwt_view")

    def device_bwt_ptr(self) -> int:
        p = c_void_p()
        check(lib().fm_device_bwt(self._h, byref(p)), "device_bwt")
        return int(p.value or 0)

    def device_struct(self, which: int):
        """(device pointer, bytes) of one index structure (fm_device_struct:
        0 BWT, 1 E, 2 transition table, 3 range-bitmap cache, 4 first wavelet
        level); (0, 0) when it is not built.  Measurement only."""
        p, b = c_void_p(), c_uint64()
        check(lib().fm_device_struct(self._h, which, byref(p), byref(b)), "device_struct")
        return int(p.value or 0), int(b.value)

    def synchronize(self) -> None:
        check(lib().fm_synchronize(self._h), "synchronize")


def load_FMIndex(path: str, device: Optional[int] = None, options=None) -> FMIndex:
    """fm_index.cpp:201-209: this engine's own file (csrc/fileformat.h), or a
    reference ``.fmi`` (sdsl csa_wt_int<> serialisation, fmidx/sdsl_fmi.py --
    parity unpinned: no sdsl file exists to test against).  ``options``: the
    index structures to build (as FMIndex's)."""
    from .options import as_build_options
    from .sdsl_fmi import is_sdsl_file, load_sdsl_fmi

    if os.path.isfile(path) and is_sdsl_file(path):
        return load_sdsl_fmi(path, device, options=options)
    o = as_build_options(options)
    obj = FMIndex.__new__(FMIndex)
    obj._h = c_void_p()
    obj._device = _default_device() if device is None else int(device)
    check(lib().fm_load_ex(byref(obj._h), str(path).encode(), obj._device, byref(o) if o is not None else None),
          "load_FMIndex")
    return obj


__all__ = ["FMIndex", "load_FMIndex", "FMIndexError", "suffix_sort_device", "wt_int_levels_device"]


def suffix_sort_device(text, want_sa: bool = False):
    """GPU suffix sorting of T' (int32 CUDA tensor, unique sentinel 0 last):
    returns (bwt int32, sa int64 or None) on the same device."""
    import torch

    assert text.is_cuda and text.dtype == torch.int32 and text.is_contiguous()
    n = text.numel()
    bwt = torch.empty(n, dtype=torch.int32, device=text.device)
    sa = torch.empty(n, dtype=torch.int64, device=text.device) if want_sa else None
    with torch.cuda.device(text.device):
        check(lib().fm_suffix_sort_device(c_void_p(text.data_ptr()), n, c_void_p(bwt.data_ptr()),
                                          c_void_p(sa.data_ptr()) if sa is not None else None,
                                          c_void_p(_stream_of(text))), "suffix_sort_device")
    return bwt, sa


def wt_int_levels_device(bwt, L: int):
    """sdsl wt_int level bit vectors of a device BWT: int64 tensor [L, ceil(n/64)]
    (bit patterns of uint64 words, LSB-first)."""
    import torch

    assert bwt.is_cuda and bwt.dtype == torch.int32 and bwt.is_contiguous()
    n = bwt.numel()
    words = torch.empty((L, (n + 63) // 64), dtype=torch.int64, device=bwt.device)
    with torch.cuda.device(bwt.device):
        check(lib().fm_wt_int_levels_device(c_void_p(bwt.data_ptr()), n, int(L), c_void_p(words.data_ptr()),
                                            c_void_p(_stream_of(bwt))), "wt_int_levels_device")
    return words
