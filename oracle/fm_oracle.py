"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This module is the checker for the MI355X FM-index engine.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product path (``fm-index-constrained-decoding_amd/``) never does.

It is a naive, obviously-correct restatement of the reference's hot path:

* ``NaiveFMIndex`` restates the SWIG surface of
  ``cpp_modules_linux/fm_index.cpp`` (class ``FMIndex``, lines 27-209) and the
  sdsl-lite arithmetic underneath it ([sdsl] ``csa_wt_int<>``,
  ``backward_search``, ``interval_symbols``).  sdsl-lite is not vendored in the
  reference and is absent here, so its semantics are re-derived from the
  definitions: the text T' gets a unique minimal sentinel 0 appended (sdsl
  ``construct`` / ``append_zero_symbol``), the suffix array of T' is therefore
  unique, and ranges / counts / distinct sets are fully determined by it.
  The suffix array is built by prefix doubling with ``numpy.lexsort``; rank is
  a binary search over per-symbol occurrence lists; distinct symbols come from
  ``numpy.unique``.  No wavelet structure is involved, so this shares no code
  path with the GPU engine.
* ``OracleIndex`` restates the Python layer ``index.py:20-207`` (doc
  reversal, ``SHIFT = 10``, ``beginnings``, early exit of ``get_range``,
  sentinel filtering in ``get_distinct_count``) on top of ``NaiveFMIndex``.

Parity pinning: the Python layer is pinned by golden vectors produced by
running the reference's own ``index.py`` and logits processors over this
restatement (``tests/golden/make_golden.py``); the sdsl layer is pinned by the
hand-derived known answers in ``tests/test_oracle.py`` and by the uniqueness
of the suffix array ("Oracle").
"""
from __future__ import annotations

import bisect
import json
import struct
from typing import Iterable, List, Sequence, Tuple

import numpy as np

SHIFT = 10                      # index.py:16
UINT64_MAX = (1 << 64) - 1      # (size_type)-1 returned by locate, fm_index.cpp:170


# --------------------------------------------------------------------------
# suffix array / BWT (definition-level, O(n log^2 n))
# --------------------------------------------------------------------------
def suffix_array(text: np.ndarray) -> np.ndarray:
    """SA of ``text`` (which must end in a unique minimal sentinel)."""
    n = int(text.shape[0])
    if n == 0:
        return np.zeros(0, dtype=np.int64)
    _, rank = np.unique(text.astype(np.int64), return_inverse=True)
    rank = rank.astype(np.int64)
    h = 1
    while True:
        second = np.full(n, -1, dtype=np.int64)
        if h < n:
            second[: n - h] = rank[h:]
        sa = np.lexsort((second, rank))
        r1 = rank[sa]
        r2 = second[sa]
        head = np.empty(n, dtype=bool)
        head[0] = True
        head[1:] = (r1[1:] != r1[:-1]) | (r2[1:] != r2[:-1])
        new = np.cumsum(head) - 1
        rank = np.empty(n, dtype=np.int64)
        rank[sa] = new
        if new[-1] == n - 1:
            return sa.astype(np.int64)
        h *= 2


class NaiveFMIndex:
    """Restatement of ``FMIndex`` in ``cpp_modules_linux/fm_index.hpp:20-45``."""

    def __init__(self):
        self._n = 0
        self._text = np.zeros(0, dtype=np.int64)

    # -- construction ------------------------------------------------------
    def initialize(self, data: Sequence[int]) -> None:
        """fm_index.cpp:33-41 (sdsl ``construct_im``: append sentinel 0)."""
        self._initialize_data(data)

    def _initialize_data(self, data: Sequence[int]) -> None:
        arr = np.asarray(list(data), dtype=np.int64)
        if arr.size and int(arr.min()) <= 0:
            raise ValueError("text contains 0 symbol (sdsl construct rejects it)")
        self._build(np.concatenate([arr, np.zeros(1, dtype=np.int64)]))

    def initialize_from_file(self, path: str, width: int) -> None:
        """fm_index.cpp:43-48: little-endian integers of ``width`` bytes."""
        raw = open(path, "rb").read()
        dt = {1: "<u1", 2: "<u2", 4: "<u4", 8: "<u8"}[int(width)]
        self._initialize_data(np.frombuffer(raw, dtype=dt).astype(np.int64).tolist())

    def _build(self, text: np.ndarray) -> None:
        self._text = text
        self._n = n = int(text.shape[0])
        self._sa = suffix_array(text)
        self._isa = np.empty(n, dtype=np.int64)
        self._isa[self._sa] = np.arange(n, dtype=np.int64)
        self._bwt = text[(self._sa - 1) % n]
        syms, counts = np.unique(self._bwt, return_counts=True)
        self._syms = syms
        self._C = {}
        run = 0
        for s, c in zip(syms.tolist(), counts.tolist()):
            self._C[s] = run
            run += c
        # per-symbol sorted occurrence positions (stable argsort keeps them ascending)
        order = np.argsort(self._bwt, kind="stable")
        sorted_bwt = self._bwt[order]
        starts = np.searchsorted(sorted_bwt, syms, side="left")
        ends = np.searchsorted(sorted_bwt, syms, side="right")
        self._occ = {}
        for s, a, b in zip(syms.tolist(), starts.tolist(), ends.tolist()):
            self._occ[s] = order[a:b]

    # -- primitives --------------------------------------------------------
    def size(self) -> int:
        return self._n

    def rank(self, i: int, c: int) -> int:
        """occurrences of ``c`` in BWT[0:i)."""
        occ = self._occ.get(int(c))
        if occ is None:
            return 0
        return int(np.searchsorted(occ, i, side="left"))

    def _sdsl_backward_search(self, l: int, r: int, c: int) -> Tuple[int, int]:
        """[sdsl] backward_search on an inclusive range, unsigned 64-bit."""
        if c not in self._C:
            if c > 0:
                return 1, 0
        cb = self._C.get(c, 0)
        lr = (cb + self.rank(l, c)) & UINT64_MAX
        rr = (cb + self.rank(r + 1, c) - 1) & UINT64_MAX
        return lr, rr

    def backward_search_step(self, symbol: int, low: int, high: int) -> Tuple[int, int]:
        """fm_index.cpp:67-97: inclusive ``high`` in, half-open out, empty -> (0,0)."""
        n = self._n
        if high >= n:
            high = n - 1
        if low > high:
            return (0, 0)
        nl, nh = self._sdsl_backward_search(low, high, symbol)
        if nl > nh:
            return (0, 0)
        return (nl, (nh + 1) & UINT64_MAX)

    def backward_search_multi(self, query: Sequence[int]) -> Tuple[int, int]:
        """fm_index.cpp:55-65: no early exit, no empty mapping."""
        l, r = 0, self._n - 1
        for c in query:
            if l > r:
                # sdsl asserts l <= r; the reference is built without NDEBUG,
                # so this is undefined territory.  Continue arithmetically.
                pass
            l, r = self._sdsl_backward_search(l, r, int(c))
        return (l, (r + 1) & UINT64_MAX)

    def _interval(self, low: int, high: int):
        if low == high:
            return None
        if high > self._n:
            high = self._n
        if low >= high:
            return None
        return np.unique(self._bwt[low:high], return_counts=True)

    def distinct(self, low: int, high: int) -> Tuple[int, ...]:
        """fm_index.cpp:99-117."""
        res = self._interval(low, high)
        if res is None:
            return tuple()
        return tuple(int(x) for x in res[0])

    def distinct_count(self, low: int, high: int) -> Tuple[int, ...]:
        """fm_index.cpp:119-144: interleaved (symbol, count), ascending symbols."""
        res = self._interval(low, high)
        if res is None:
            return tuple()
        out: List[int] = []
        for s, c in zip(res[0].tolist(), res[1].tolist()):
            out.append(int(s))
            out.append(int(c))
        return tuple(out)

    def distinct_count_multi(self, lows: Sequence[int], highs: Sequence[int]):
        """fm_index.cpp:146-166: results in input order."""
        return tuple(self.distinct_count(int(a), int(b)) for a, b in zip(lows, highs))

    def locate(self, row: int) -> int:
        """fm_index.cpp:168-172."""
        if row >= self._n:
            return UINT64_MAX
        return int(self._sa[row])

    def extract_text(self, begin: int, end: int) -> Tuple[int, ...]:
        """fm_index.cpp:174-194 (LF walk from isa[end-1])."""
        if end <= begin:
            return tuple()
        if end > self._n:
            end = self._n
        if end <= begin:
            # fm_index.cpp:184 loops (end-begin-1) times in unsigned arithmetic:
            # unbounded in the reference, rejected here.
            raise ValueError("extract_text: begin >= clamped end")
        start = int(self._isa[end - 1])
        sym = int(self._bwt[start])
        ret = [sym]
        if end - begin == 1:
            return tuple(ret)
        for _ in range(end - begin - 1):
            start = self.backward_search_step(sym, start, start + 1)[0]
            if start >= self._n:
                break
            sym = int(self._bwt[start])
            ret.append(sym)
        return tuple(ret)

    # -- persistence (oracle-private format, not sdsl's) ------------------
    def save(self, path: str) -> None:
        np.save(path if path.endswith(".npy") else path + ".npy", self._text)

    @property
    def bwt(self) -> np.ndarray:
        return self._bwt

    @property
    def sa(self) -> np.ndarray:
        return self._sa

    @property
    def text(self) -> np.ndarray:
        return self._text


def load_naive(path: str) -> NaiveFMIndex:
    fm = NaiveFMIndex()
    fm._build(np.load(path if path.endswith(".npy") else path + ".npy"))
    return fm


# --------------------------------------------------------------------------
# index.py restatement
# --------------------------------------------------------------------------
def encode_corpus(sequences: Iterable[Sequence[int]]):
    """index.py:47-53: docs reversed, ids + SHIFT, concatenated, no separators."""
    beginnings = [0]
    occurring = set()
    data: List[int] = []
    for seq in sequences:
        seq = list(seq)
        beginnings.append(beginnings[-1] + len(seq))
        occurring |= set(seq)
        data.extend(x + SHIFT for x in seq[::-1])
    return data, beginnings, occurring


class OracleIndex(NaiveFMIndex):
    """Restatement of ``index.FMIndex`` (index.py:20-207)."""

    def __init__(self):
        super().__init__()
        self.beginnings = [0]
        self.occurring = set()
        self.occurring_distinct: List[int] = []
        self.occurring_counts: List[int] = []
        self.labels = None

    def initialize(self, sequences, in_memory: bool = False) -> None:  # type: ignore[override]
        data, beginnings, occurring = encode_corpus(sequences)
        self.beginnings = beginnings
        self.occurring = list(occurring)
        NaiveFMIndex.initialize(self, data)
        # index.py:67 -- len(self) == beginnings[-1] == size()-1: the last BWT row is excluded
        self.occurring_distinct, self.occurring_counts = self.get_distinct_count(0, len(self))

    def __len__(self) -> int:
        return self.beginnings[-1]

    @property
    def n_docs(self) -> int:
        return len(self.beginnings) - 1

    def get_range(self, sequence: Sequence[int]) -> Tuple[int, int]:
        """index.py:103-114 -- early exit on (0, 0)."""
        lo, hi = 0, self.size()
        for tok in sequence:
            lo, hi = self.backward_search_step(int(tok) + SHIFT, lo, hi - 1)
            if lo == hi == 0:
                return lo, hi
        return lo, hi

    def get_count(self, sequence: Sequence[int]) -> int:
        lo, hi = self.get_range(sequence)
        return hi - lo

    def get_distinct(self, low: int, high: int) -> List[int]:
        return [c - SHIFT for c in self.distinct(low, high) if c > 0]

    def get_distinct_count(self, low: int, high: int):
        data = self.distinct_count(low, high)
        syms = [d - SHIFT for d, c in zip(data[0::2], data[1::2]) if d > 0]
        cnts = [c for d, c in zip(data[0::2], data[1::2]) if d > 0]
        return syms, cnts

    def get_distinct_count_multi(self, lows, highs):
        out = []
        for data in self.distinct_count_multi(lows, highs):
            syms = [d - SHIFT for d, c in zip(data[0::2], data[1::2]) if d > 0]
            cnts = [c for d, c in zip(data[0::2], data[1::2]) if d > 0]
            out.append((syms, cnts))
        return out

    def get_continuations(self, sequence):
        lo, hi = self.get_range(sequence)
        return self.get_distinct(lo, hi)

    def get_doc(self, doc_index: int) -> List[int]:
        doc = self.extract_text(self.beginnings[doc_index], self.beginnings[doc_index + 1])
        return [x - SHIFT for x in doc]

    def get_doc_index(self, token_index: int) -> int:
        return bisect.bisect_right(self.beginnings, token_index) - 1

    def get_doc_length(self, doc_index: int) -> int:
        return self.beginnings[doc_index + 1] - self.beginnings[doc_index]

    def get_token_index_from_row(self, row: int) -> int:
        return self.locate(row)

    def get_doc_index_from_row(self, row: int) -> int:
        return self.get_doc_index(self.locate(row))

    def get_doc_indices(self, sequence):
        lo, hi = self.get_range(sequence)
        for row in range(lo, hi):
            yield self.get_doc_index_from_row(row)


# --------------------------------------------------------------------------
# helpers used by tests / bench (mask view of the hot path)
# --------------------------------------------------------------------------
def allowed_mask(fm: NaiveFMIndex, lows, highs, vocab: int, shift: int = SHIFT) -> np.ndarray:
    """Boolean core of every processor: allowed[b, t] = 1 iff
    t + shift occurs in BWT[low_b, high_b)."""
    out = np.zeros((len(lows), vocab), dtype=np.uint8)
    for b, (lo, hi) in enumerate(zip(lows, highs)):
        if hi > fm.size():
            hi = fm.size()
        if lo >= hi:
            continue
        syms = np.unique(fm.bwt[lo:hi]) - shift
        syms = syms[(syms >= 0) & (syms < vocab)]
        out[b, syms] = 1
    return out


def wm_node_count(fm: NaiveFMIndex, lo: int, hi: int, levels: int) -> int:
    """Non-empty wavelet nodes below the root visited by an interval
    enumeration of BWT[lo, hi): sum over levels 1..L of distinct symbol
    prefixes present (N_nodes)."""
    if lo >= hi:
        return 0
    syms = np.unique(fm.bwt[lo:hi]).astype(np.int64)
    total = 0
    for depth in range(1, levels + 1):
        total += int(np.unique(syms >> (levels - depth)).shape[0])
    return total


def dump_json(obj, path: str) -> None:
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"))


def pack_int32_le(data: Sequence[int]) -> bytes:
    """index.py:63 packs each symbol with struct format '<l'."""
    return b"".join(struct.pack("<l", int(x)) for x in data)
