"""Reader of the reference's own on-disk index: the ``.fmi`` file that
``FMIndex::save`` writes with sdsl ``store_to_file`` and ``load_FMIndex``
reads with ``load_from_file`` (cpp_modules_linux/fm_index.cpp:196-209;
index.py:197-207 opens ``path + '.fmi'``), i.e. sdsl-lite's serialisation of
``csa_wt_int<>`` = ``csa_wt<wt_int<>, 32, 64, sa_order_sa_sampling<>,
isa_sampling<>, int_alphabet<>>``.

PARITY UNPINNED.  sdsl-lite is not vendored in the reference, cannot be built
offline, and no ``.fmi`` file exists in the reference or this environment, so
the layout below is restated from sdsl-lite's ``serialize()`` member order and
is tested only against this repository's own writer of the same layout
(tests/sdsl_writer.py) -- a round trip, not a reference file.  The reader
validates everything it can from the file itself (sizes, widths, the alphabet's
C array against the decoded symbol counts, every ISA sample against the BWT's
LF walks, and the SA samples against locate), so a layout mismatch on a real
sdsl file fails loudly instead of yielding a wrong index.

Layout read (little endian, sdsl-lite 2.x):

* ``bit_vector`` / ``int_vector<64>``: size in bits (u64), then
  ceil(size / 64) u64 words.
* ``int_vector<0>``: size in bits (u64), width (u8), then ceil(size / 64) u64
  words; element i occupies bits [i w, (i + 1) w), LSB first.
* ``rank_support_v``: its directory (an ``int_vector<64>``).
* ``select_support_mcl``: arg_cnt (u64); if arg_cnt > 0: superblock
  (``int_vector<0>``), mini_or_long (``bit_vector``), then one
  ``int_vector<0>`` per superblock of 4096 ones (long superblock or
  miniblock).  Skipped: the reader needs no select.
* ``wt_int``: size (u64), sigma (u64), tree (``bit_vector`` of size * max_level
  bits: level l at bits [l size, (l + 1) size), the sequence stably sorted by
  its top l bits, bit (max_level - 1 - l) of each symbol), tree_rank,
  tree_select1, tree_select0, max_level (u32), zero_cnt and rank_level
  (``int_vector<64>``, max_level entries each).
* ``csa_wt``: wavelet tree (over the compact alphabet), sa samples (SA[32 i]),
  isa samples (ISA[64 k] = the row of text position 64 k), alphabet.
* ``int_alphabet``: char (``bit_vector``, empty when the alphabet is
  0 .. sigma - 1), char_rank, char_select, C (``int_vector<64>``, sigma + 1),
  sigma (u64).

Conversion: the wavelet tree is inverted on the GPU (torch, one pass per
level: ~40 bytes of device memory per row at peak) into the compact BWT,
mapped through the alphabet to T' symbols (token id + 10, sentinel 0), handed
to ``fm_initialize_from_bwt_device``; the ISA samples then give locate /
extract through ``fm_attach_isa_samples_device`` (every sample checked by an LF
walk), and the file's SA samples are compared with ``locate`` of their rows.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

SDSL_SA_RATE = 32
SDSL_ISA_RATE = 64


class SdslFormatError(ValueError):
    """The file does not parse as sdsl's csa_wt_int<> serialisation."""


class _Cursor:
    def __init__(self, buf: np.ndarray, path: str):
        self.b = buf
        self.p = 0
        self.path = path

    def need(self, k: int, what: str):
        if self.p + k > self.b.size:
            raise SdslFormatError(f"{self.path}: truncated inside {what} (offset {self.p}, need {k} bytes)")

    def u64(self, what: str) -> int:
        self.need(8, what)
        v = int(self.b[self.p:self.p + 8].view(np.uint64)[0])
        self.p += 8
        return v

    def u32(self, what: str) -> int:
        self.need(4, what)
        v = int(self.b[self.p:self.p + 4].view(np.uint32)[0])
        self.p += 4
        return v

    def u8(self, what: str) -> int:
        self.need(1, what)
        v = int(self.b[self.p])
        self.p += 1
        return v

    def words(self, nbits: int, what: str) -> np.ndarray:
        nw = (nbits + 63) // 64
        self.need(8 * nw, what)
        w = self.b[self.p:self.p + 8 * nw].view(np.uint64)
        self.p += 8 * nw
        return w

    def bit_vector(self, what: str, max_bits: int):
        size = self.u64(what)
        if size > max_bits:
            raise SdslFormatError(f"{self.path}: {what} of {size} bits is implausible")
        return size, self.words(size, what)

    def int_vector0(self, what: str, max_bits: int):
        size = self.u64(what)
        width = self.u8(what)
        if not 1 <= width <= 64 or size % width or size > max_bits:
            raise SdslFormatError(f"{self.path}: {what}: size {size} bits, width {width}")
        return size // width, width, self.words(size, what)

    def int_vector64(self, what: str, max_bits: int) -> np.ndarray:
        size = self.u64(what)
        if size % 64 or size > max_bits:
            raise SdslFormatError(f"{self.path}: {what}: {size} bits is not a whole number of u64")
        return self.words(size, what)

    def skip_select_mcl(self, what: str, max_bits: int):
        arg_cnt = self.u64(what)
        if arg_cnt == 0:
            return
        sb = (arg_cnt + 4095) >> 12
        self.int_vector0(what + ".superblock", max_bits)
        mol_bits, _ = self.bit_vector(what + ".mini_or_long", max_bits)
        if mol_bits not in (0, sb):
            raise SdslFormatError(f"{self.path}: {what}: mini_or_long of {mol_bits} bits for {sb} superblocks")
        for _ in range(sb):
            self.int_vector0(what + ".block", max_bits)


def unpack_int_vector(words: np.ndarray, count: int, width: int) -> np.ndarray:
    """Elements of an int_vector<0> (LSB-first packing across u64 words)."""
    if count == 0:
        return np.zeros(0, dtype=np.uint64)
    w = np.concatenate([words.astype(np.uint64), np.zeros(1, dtype=np.uint64)])
    bit = np.arange(count, dtype=np.uint64) * np.uint64(width)
    wi = (bit >> np.uint64(6)).astype(np.int64)
    off = bit & np.uint64(63)
    lo = w[wi] >> off
    # bits from the next word (off + width > 64); shifting by 64 is undefined, so mask it out
    sh = (np.uint64(64) - off) & np.uint64(63)
    hi = np.where(off == 0, np.uint64(0), w[wi + 1] << sh)
    mask = np.uint64((1 << width) - 1) if width < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    return (lo | hi) & mask


class SdslCsaWtInt:
    """The parsed pieces of a csa_wt_int<> file (host arrays, not yet decoded)."""

    def __init__(self, path: str):
        buf = np.fromfile(path, dtype=np.uint8)
        c = _Cursor(buf, path)
        cap = 8 * buf.size                     # no structure can hold more bits than the file
        # ---- wt_int
        self.n = c.u64("wt_int.size")
        self.wt_sigma = c.u64("wt_int.sigma")
        if self.n == 0 or self.n >= (1 << 34):
            raise SdslFormatError(f"{path}: wt_int size {self.n} out of range (0 < n < 2^34)")
        tree_bits, self.tree = c.bit_vector("wt_int.tree", cap)
        c.int_vector64("wt_int.tree_rank", cap)
        c.skip_select_mcl("wt_int.tree_select1", cap)
        c.skip_select_mcl("wt_int.tree_select0", cap)
        save = c.p
        self.max_level = None
        for width in (4, 8):       # u32 in sdsl-lite 2.x; a u64 variant is accepted if it is the one that parses
            c.p = save
            L = c.u32("wt_int.max_level") if width == 4 else c.u64("wt_int.max_level")
            if L == 0 or L > 64 or L * self.n != tree_bits:
                continue
            try:
                z = c.int_vector64("wt_int.zero_cnt", cap)
                r = c.int_vector64("wt_int.rank_level", cap)
            except SdslFormatError:
                continue
            if z.size == L and r.size == L:
                self.max_level = L
                self.zero_cnt = z.copy()
                break
        if self.max_level is None:
            raise SdslFormatError(f"{path}: wt_int max_level / zero_cnt do not match a tree of {tree_bits} bits "
                                  f"over {self.n} rows")
        # ---- samples
        cnt, width, words = c.int_vector0("sa_samples", cap)
        if cnt != (self.n + SDSL_SA_RATE - 1) // SDSL_SA_RATE:
            raise SdslFormatError(f"{path}: {cnt} SA samples for n = {self.n}")
        self.sa_samples = unpack_int_vector(words, cnt, width)
        cnt, width, words = c.int_vector0("isa_samples", cap)
        if cnt != (self.n - 1) // SDSL_ISA_RATE + 1:
            raise SdslFormatError(f"{path}: {cnt} ISA samples for n = {self.n}")
        self.isa_samples = unpack_int_vector(words, cnt, width)
        # ---- int_alphabet
        char_bits, char_words = c.bit_vector("alphabet.char", cap)
        c.int_vector64("alphabet.char_rank", cap)
        c.skip_select_mcl("alphabet.char_select", cap)
        self.C = c.int_vector64("alphabet.C", cap).copy()
        self.sigma = c.u64("alphabet.sigma")
        if c.p != buf.size:
            raise SdslFormatError(f"{path}: {buf.size - c.p} trailing bytes after the alphabet")
        if self.C.size != self.sigma + 1 or int(self.C[-1]) != self.n or np.any(np.diff(self.C.astype(np.int64)) < 0):
            raise SdslFormatError(f"{path}: alphabet C array inconsistent with sigma {self.sigma} / n {self.n}")
        if self.wt_sigma != self.sigma:
            raise SdslFormatError(f"{path}: wavelet tree sigma {self.wt_sigma} != alphabet sigma {self.sigma}")
        if char_bits:
            bits = np.unpackbits(char_words.view(np.uint8), bitorder="little")[:char_bits]
            self.comp2char = np.flatnonzero(bits).astype(np.int64)
        else:
            self.comp2char = np.arange(self.sigma, dtype=np.int64)
        if self.comp2char.size != self.sigma:
            raise SdslFormatError(f"{path}: alphabet has {self.comp2char.size} characters, sigma {self.sigma}")
        if self.sigma and (self.max_level < max(1, int(self.sigma - 1).bit_length())):
            raise SdslFormatError(f"{path}: {self.max_level} levels cannot hold {self.sigma} symbols")


def decode_wt_int_device(tree_words: np.ndarray, n: int, L: int, device, chunk: int = 1 << 27):
    """The sequence a wt_int tree encodes (compact symbols, int64 [n] on
    ``device``), by one pass per level: every position carries its prefix
    (the symbol's top l bits) and its position in level l's order; level l's
    bit there is the next bit, and the position in level l + 1's order is its
    node's start + its rank among the node's zeros (or the node's zero count +
    its rank among the ones) -- node starts from the prefix counts, ranks from
    one cumulative sum of the level's zeros."""
    import torch

    tw = torch.from_numpy(np.ascontiguousarray(tree_words).view(np.int64)).to(device)
    pos = torch.arange(n, dtype=torch.int64, device=device)
    val = torch.zeros(n, dtype=torch.int64, device=device)
    for lev in range(L):
        # level bits in level order (bit lev * n + j of the tree), chunked
        bits = torch.empty(n, dtype=torch.uint8, device=device)
        for a in range(0, n, chunk):
            j = torch.arange(a, min(n, a + chunk), dtype=torch.int64, device=device) + lev * n
            bits[a:a + j.numel()] = ((tw[j >> 6] >> (j & 63)) & 1).to(torch.uint8)
            del j
        cz = torch.zeros(n + 1, dtype=torch.int64, device=device)
        torch.cumsum(1 - bits.to(torch.int64), 0, out=cz[1:])
        cnt = torch.bincount(val, minlength=1 << lev) if lev else torch.tensor([n], device=device)
        start = torch.zeros(cnt.numel() + 1, dtype=torch.int64, device=device)
        torch.cumsum(cnt, 0, out=start[1:])
        ns = start[val]
        ne = start[val + 1]
        b = bits[pos].to(torch.int64)
        zb = cz[pos] - cz[ns]
        zn = cz[ne] - cz[ns]
        pos = torch.where(b == 0, ns + zb, ns + zn + (pos - ns) - zb)
        val = val * 2 + b
        del bits, cz, cnt, start, ns, ne, b, zb, zn
    return val


def load_sdsl_fmi(path: str, device: Optional[int] = None, verify_samples: bool = True):
    """An engine FMIndex (fmidx.fm_index.FMIndex, the SWIG surface) from a
    reference ``.fmi`` file (see the module docstring; parity unpinned)."""
    import torch

    from ._lib import check, lib
    from .fm_index import FMIndex, _default_device, _stream_of
    from ctypes import c_void_p

    f = SdslCsaWtInt(path)
    dev_index = _default_device() if device is None else int(device)
    dev = torch.device("cuda", dev_index)
    comp = decode_wt_int_device(f.tree, f.n, f.max_level, dev)
    counts = torch.bincount(comp, minlength=int(f.sigma)).cpu().numpy()
    if counts.size != f.sigma or not np.array_equal(counts.astype(np.uint64), np.diff(f.C)):
        raise SdslFormatError(f"{path}: decoded wavelet tree disagrees with the alphabet's C array")
    bwt = torch.from_numpy(f.comp2char).to(dev)[comp].to(torch.int32)
    del comp
    if int((bwt == 0).sum()) != 1:
        raise SdslFormatError(f"{path}: the decoded BWT must hold exactly one sentinel 0")
    ix = FMIndex(device=dev_index)
    ix.initialize_from_bwt_device(bwt)
    del bwt
    isa = torch.from_numpy(f.isa_samples.view(np.int64)).to(dev)
    check(lib().fm_attach_isa_samples_device(ix._h, c_void_p(isa.data_ptr()), isa.numel(),
                                             c_void_p(_stream_of(isa))), "attach_isa_samples")
    if verify_samples:
        rows = torch.arange(0, f.n, SDSL_SA_RATE, dtype=torch.int64, device=dev)
        got = ix.locate_batch(rows)
        want = torch.from_numpy(f.sa_samples.view(np.int64)).to(dev)
        if not torch.equal(got, want):
            raise SdslFormatError(f"{path}: the file's SA samples disagree with locate on the decoded index")
    return ix


def is_sdsl_file(path: str) -> bool:
    """True unless the file starts with this engine's own magic (fileformat.h)."""
    with open(path, "rb") as fh:
        return fh.read(8) != b"FMIDXAMD"


__all__ = ["SdslCsaWtInt", "SdslFormatError", "decode_wt_int_device", "load_sdsl_fmi", "is_sdsl_file",
           "unpack_int_vector"]
