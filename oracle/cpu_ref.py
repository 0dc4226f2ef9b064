"""ctypes wrapper of oracle/_build/libcpuref.so -- TEST INFRASTRUCTURE ONLY
(the sdsl-faithful CPU restatement used as checker and as the bench's
cpu_baseline).  See cpu_ref.cpp for what it restates."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_int, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libcpuref.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run `make -C oracle`")
        d = ctypes.CDLL(LIB)
        u64p = POINTER(c_uint64)
        d.cr_build.restype = c_void_p
        d.cr_build.argtypes = [u64p, c_uint64, c_uint32, u64p, c_uint64]
        d.cr_free.argtypes = [c_void_p]
        d.cr_backward_search_step.argtypes = [c_void_p, c_uint64, c_uint64, c_uint64, u64p]
        d.cr_distinct_count.restype = c_uint64
        d.cr_distinct_count.argtypes = [c_void_p, c_uint64, c_uint64, u64p, c_uint64]
        d.cr_decode_step.argtypes = [c_void_p, POINTER(c_int64), c_int64, c_int64, u64p, u64p, c_uint64,
                                     POINTER(ctypes.c_uint8), c_uint64, c_int]
        d.cr_distinct_only.argtypes = [c_void_p, u64p, u64p, c_uint64, c_int]
        d.cr_decode_step_timed.argtypes = [c_void_p, POINTER(c_int64), c_int64, c_int64, u64p, u64p, c_uint64,
                                           POINTER(ctypes.c_uint8), c_uint64, c_int, POINTER(ctypes.c_double)]
        d.cr_full_step.argtypes = [c_void_p, POINTER(c_int64), POINTER(c_int64), c_int64, c_uint64, u64p, u64p,
                                   POINTER(ctypes.c_uint8), c_uint64, c_int, c_int]
        _lib = d
    return _lib


def _p(a, t=c_uint64):
    return a.ctypes.data_as(POINTER(t))


def levels_numpy(bwt: np.ndarray, L: int) -> np.ndarray:
    """wt_int level bit vectors: level l = BWT stably sorted by its top l bits."""
    n = bwt.size
    wpl = (n + 63) // 64
    out = np.zeros((L, wpl), dtype=np.uint64)
    b = bwt.astype(np.int64)
    for lev in range(L):
        seq = b if lev == 0 else b[np.argsort(b >> (L - lev), kind="stable")]
        bits = ((seq >> (L - 1 - lev)) & 1).astype(np.uint8)
        packed = np.packbits(bits, bitorder="little")
        buf = np.zeros(wpl * 8, dtype=np.uint8)
        buf[: packed.size] = packed
        out[lev] = buf.view(np.uint64)
    return out


def c_array(bwt: np.ndarray, L: int) -> np.ndarray:
    cnt = np.bincount(bwt.astype(np.int64), minlength=(1 << L) + 1).astype(np.uint64)
    C = np.zeros((1 << L) + 1, dtype=np.uint64)
    np.cumsum(cnt[: 1 << L], out=C[1:])
    return C


class CpuRef:
    def __init__(self, level_words: np.ndarray, n: int, L: int, C: np.ndarray, sigma: int):
        self.n = n
        self.L = L
        lw = np.ascontiguousarray(level_words, dtype=np.uint64)
        Cc = np.ascontiguousarray(C, dtype=np.uint64)
        self._h = lib().cr_build(_p(lw), n, L, _p(Cc), sigma)

    @classmethod
    def from_bwt(cls, bwt: np.ndarray) -> "CpuRef":
        bwt = np.asarray(bwt)
        L = max(1, int(bwt.max()).bit_length())
        return cls(levels_numpy(bwt, L), bwt.size, L, c_array(bwt, L), int(np.unique(bwt).size))

    @classmethod
    def from_device_bwt(cls, bwt) -> "CpuRef":
        """From a device BWT at any scale: the wt_int level vectors are built on
        the GPU (fm_wt_int_levels_device, itself checked against
        levels_numpy) and copied to the host; C / sigma by bincount."""
        import torch

        from fmidx.fm_index import wt_int_levels_device

        n = bwt.numel()
        L = max(1, int(bwt.max().item()).bit_length())
        words = wt_int_levels_device(bwt, L).cpu().numpy().view(np.uint64)
        # symbol counts in chunks (an int64 copy of a 4.5e9-row BWT would take 36 GB of HBM)
        cnt = torch.zeros((1 << L) + 1, dtype=torch.int64, device=bwt.device)
        for a in range(0, n, 1 << 28):
            cnt += torch.bincount(bwt[a:a + (1 << 28)].to(torch.int64), minlength=(1 << L) + 1)
        C = torch.zeros((1 << L) + 1, dtype=torch.int64, device=bwt.device)
        torch.cumsum(cnt[: 1 << L], 0, out=C[1:])
        sigma = int((cnt > 0).sum().item())
        return cls(words, n, L, C.cpu().numpy().view(np.uint64), sigma)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().cr_free(self._h)
            self._h = None

    def backward_search_step(self, c, low, high):
        out = np.zeros(2, dtype=np.uint64)
        lib().cr_backward_search_step(self._h, c, low, high, _p(out))
        return int(out[0]), int(out[1])

    def distinct_count(self, low, high):
        cap = 2 * max(1, min(max(0, min(high, self.n) - low), 1 << self.L))
        out = np.zeros(cap, dtype=np.uint64)
        k = lib().cr_distinct_count(self._h, low, high, _p(out), cap)
        return tuple(int(x) for x in out[: 2 * k])

    def decode_step(self, tok: np.ndarray, shift: int, reset_below: int, lo: np.ndarray, hi: np.ndarray,
                    mask: np.ndarray, threads: int):
        lib().cr_decode_step(self._h, _p(tok, c_int64), shift, reset_below, _p(lo), _p(hi), lo.size,
                             _p(mask, ctypes.c_uint8), mask.shape[1], threads)

    def decode_step_timed(self, tok: np.ndarray, shift: int, reset_below: int, lo: np.ndarray, hi: np.ndarray,
                          mask: np.ndarray) -> float:
        """decode_step on one thread; returns the seconds its distinct_count calls took."""
        t = ctypes.c_double(0.0)
        lib().cr_decode_step_timed(self._h, _p(tok, c_int64), shift, reset_below, _p(lo), _p(hi), lo.size,
                                   _p(mask, ctypes.c_uint8), mask.shape[1], 1, ctypes.byref(t))
        return t.value

    def distinct_only(self, lo: np.ndarray, hi: np.ndarray, threads: int = 1):
        """distinct_count of every (lo[i], hi[i]) with the results discarded."""
        lo = np.ascontiguousarray(lo, dtype=np.uint64)
        hi = np.ascontiguousarray(hi, dtype=np.uint64)
        lib().cr_distinct_only(self._h, _p(lo), _p(hi), lo.size, threads)

    def full_step(self, tokens: np.ndarray, offsets: np.ndarray, shift: int, lo, hi, mask, threads: int,
                  faithful: bool = False):
        """get_range of every row's whole pattern + distinct_count + mask row;
        ``faithful`` also makes the Qwen processor's two extra searches per row."""
        lib().cr_full_step(self._h, _p(tokens, c_int64), _p(offsets, c_int64), shift, lo.size, _p(lo), _p(hi),
                           _p(mask, ctypes.c_uint8), mask.shape[1], threads, 1 if faithful else 0)
