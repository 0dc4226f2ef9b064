"""``FMIndex`` -- the ``index.py`` surface on the MI355X engine.

Reference: ``index.py:20-207``.  Same attributes (``beginnings``,
``occurring``, ``occurring_distinct``, ``occurring_counts``, ``labels``),
methods and return shapes, same corpus encoding (each doc reversed, ids +
``SHIFT``, concatenated without separators) so ranges, counts and distinct
sets are identical to the reference's.  Differences are performance-only:
``get_range`` runs the whole pattern in one GPU launch (the reference makes
one SWIG call per token, ``index.py:109-112``) and
``get_distinct_count_multi`` is one launch for all rows (``fm_index.cpp:146``
spawns a thread per row).  ``.oth`` metadata is the reference's pickle of
``(beginnings, occurring, labels)`` (index.py:189-207), read back with an
unpickler that resolves no globals (plain lists / sets / ints / strings / None
only), so a reference-saved ``.oth`` loads and nothing in it can run code.
"""
from __future__ import annotations

import bisect
import io
import json
import pickle
from typing import Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .fm_index import FMIndex as _FMIndex
from .fm_index import _u64_vec, load_FMIndex

SHIFT = 10                      # index.py:16


def encode_corpus(sequences: Iterable[Sequence[int]]):
    """index.py:47-56 -> (T' as uint64 array, beginnings, occurring set)."""
    beginnings = [0]
    parts = []
    for seq in sequences:
        a = np.asarray(list(seq) if not isinstance(seq, np.ndarray) else seq, dtype=np.int64)
        beginnings.append(beginnings[-1] + int(a.size))
        parts.append(a[::-1] + SHIFT)
    data = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
    if data.size and int(data.min()) < 0:
        raise OverflowError("token id below -SHIFT cannot be encoded")
    occurring = set((np.unique(data) - SHIFT).tolist())    # the union of set(seq) (index.py:51)
    return data.astype(np.uint64), beginnings, occurring


class FMIndex(_FMIndex):
    """Drop-in for ``index.FMIndex`` (index.py:20)."""

    beginnings: List[int]
    occurring: List[int]
    occurring_distinct: List[int]
    occurring_counts: List[int]
    labels: Optional[List[str]]

    def __init__(self, device: Optional[int] = None, options=None):
        super().__init__(device, options=options)
        self.beginnings = [0]
        self.occurring = set()
        self.occurring_distinct = []
        self.occurring_counts = []
        self.labels = None

    def initialize(self, sequences: Iterable[List[int]], in_memory: bool = False) -> None:  # type: ignore[override]
        """index.py:39-67.  ``in_memory`` is accepted for API parity; both
        paths encode in memory (the reference's temp-file path feeds the same
        symbols through ``initialize_from_file(tmp, 4)``)."""
        data, beginnings, occurring = encode_corpus(sequences)
        self.beginnings = beginnings
        self.occurring = list(occurring)
        super().initialize(data)
        self.occurring_distinct, self.occurring_counts = self.get_distinct_count(0, len(self))

    # -- docs --------------------------------------------------------------
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

    # -- search ------------------------------------------------------------
    def get_range(self, sequence: List[int]) -> Tuple[int, int]:
        """index.py:103-114 in one launch; (0, size()) for an empty pattern."""
        seq = list(sequence)
        if seq and min(seq) + SHIFT < 0:
            raise OverflowError("in method 'FMIndex_backward_search_step', argument 2 of type 'char_type'")
        lo, hi = self.get_range_batch([seq], SHIFT)
        return int(lo[0]), int(hi[0])

    def get_ranges(self, sequences: Sequence[Sequence[int]]) -> List[Tuple[int, int]]:
        """Batched ``get_range`` for many patterns (one launch)."""
        lo, hi = self.get_range_batch(sequences, SHIFT)
        return list(zip(lo.tolist(), hi.tolist()))

    def get_count(self, sequence: List[int]) -> int:
        start, end = self.get_range(sequence)
        return end - start

    def get_doc_indices(self, sequence: List[int]) -> Iterator[int]:
        """index.py:123-129: the doc of every occurrence, in row order.  All rows
        are located in one launch (fm_locate_batch) and mapped to docs by a
        binary search of ``beginnings`` on the device."""
        start, end = self.get_range(sequence)
        if end <= start:
            return
        import torch

        dev = torch.device("cuda", self.device)
        beg = torch.tensor(self.beginnings, dtype=torch.int64, device=dev)
        chunk = 1 << 20          # rows per launch: the generator stays lazy over huge ranges
        for a in range(start, end, chunk):
            rows = torch.arange(a, min(end, a + chunk), dtype=torch.int64, device=dev)
            pos = self.locate_batch(rows)
            docs = torch.searchsorted(beg, pos, right=True) - 1      # bisect_right - 1 (get_doc_index)
            yield from docs.cpu().tolist()

    def get_docs(self, doc_indices: Sequence[int]) -> List[List[int]]:
        """get_doc (index.py:69-80) of many docs in one launch."""
        b = [self.beginnings[d] for d in doc_indices]
        e = [self.beginnings[d + 1] for d in doc_indices]
        return [[x - SHIFT for x in doc] for doc in self.extract_batch(b, e)]

    def get_continuations(self, sequence: List[int]) -> List[int]:
        start, end = self.get_range(sequence)
        return self.get_distinct(start, end)

    def get_distinct(self, low: int, high: int) -> List[int]:
        return [c - SHIFT for c in self.distinct(low, high) if c > 0]

    def get_distinct_count(self, low: int, high: int) -> Tuple[List[int], List[int]]:
        data = self.distinct_count(low, high)
        syms = data[0::2]
        cnts = data[1::2]
        keep = [i for i, d in enumerate(syms) if d > 0]          # drop the sentinel (index.py:156)
        return [syms[i] - SHIFT for i in keep], [cnts[i] for i in keep]

    def get_distinct_count_multi(self, lows: List[int], highs: List[int]) -> List[Tuple[List[int], List[int]]]:
        """index.py:161-174: per range, its symbols > 0 (the sentinel dropped)
        minus SHIFT and their counts -- filtered and shifted on the result
        arrays of the one batched launch, not per symbol in Python."""
        lo = _u64_vec(lows, "distinct_count_multi", 2)
        hi = _u64_vec(highs, "distinct_count_multi", 3)
        if lo.size != hi.size:
            raise ValueError("lows and highs differ in length")
        out, offs = self._distinct_count_multi_arrays(lo, hi)
        tot = int(offs[-1]) if offs.size else 0
        pairs = out[: 2 * tot].reshape(-1, 2)
        keep = pairs[:, 0] > 0
        syms = (pairs[keep, 0].astype(np.int64) - SHIFT).tolist()
        cnts = pairs[keep, 1].astype(np.int64).tolist()
        ko = np.concatenate([[0], np.cumsum(keep)]).astype(np.int64)[offs.astype(np.int64)].tolist()
        return [(syms[ko[i]:ko[i + 1]], cnts[ko[i]:ko[i + 1]]) for i in range(lo.size)]

    def __len__(self) -> int:
        return self.beginnings[-1]

    @property
    def n_docs(self) -> int:
        return len(self.beginnings) - 1

    # -- persistence ---------------------------------------------------------
    def save(self, path: str) -> None:  # type: ignore[override]
        """index.py:189-195: ``.oth`` = pickle of (beginnings, occurring, labels)."""
        with open(path + ".oth", "wb") as f:
            pickle.dump((list(self.beginnings), list(self.occurring), self.labels), f)
        return super().save(path + ".fmi")

    @classmethod
    def load(cls, path: str, device: Optional[int] = None, options=None) -> "FMIndex":
        """index.py:197-207 (``options``: fmidx.options build options)."""
        index = load_FMIndex(path + ".fmi", device, options=options)
        index.__class__ = cls
        index.beginnings, index.occurring, index.labels = read_oth(path + ".oth")
        index.occurring_distinct, index.occurring_counts = index.get_distinct_count(0, len(index))
        return index


class _DataOnlyUnpickler(pickle.Unpickler):
    """Unpickles builtin containers and scalars only: every global lookup
    (the only way a pickle can name code to run) is refused, except the set
    constructors that pickle protocols < 4 spell as a global."""

    _SAFE = {("builtins", "set"): set, ("builtins", "frozenset"): frozenset,
             ("__builtin__", "set"): set, ("__builtin__", "frozenset"): frozenset}

    def find_class(self, module, name):
        if (module, name) in self._SAFE:
            return self._SAFE[(module, name)]
        raise pickle.UnpicklingError(f".oth metadata may not reference {module}.{name}")


def read_oth(path: str):
    """(beginnings, occurring, labels) of a ``.oth`` file: the reference's
    pickle (index.py:194), or the JSON this engine wrote before it used pickle."""
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:1] == b"{":
        meta = json.loads(raw.decode())
        return ([int(x) for x in meta["beginnings"]], [int(x) for x in meta["occurring"]], meta.get("labels"))
    obj = _DataOnlyUnpickler(io.BytesIO(raw)).load()
    if not (isinstance(obj, tuple) and len(obj) == 3):
        raise ValueError(f"{path}: expected a (beginnings, occurring, labels) tuple")
    beginnings, occurring, labels = obj
    if not all(isinstance(x, int) for x in beginnings):
        raise ValueError(f"{path}: beginnings must be ints")
    return list(beginnings), occurring, labels


__all__ = ["FMIndex", "SHIFT", "encode_corpus", "read_oth"]
