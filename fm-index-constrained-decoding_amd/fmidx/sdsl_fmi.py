"""Reader of the reference's own on-disk index: the ``.fmi`` file that
``FMIndex::save`` writes with sdsl ``store_to_file`` and ``load_FMIndex``
reads with ``load_from_file`` (cpp_modules_linux/fm_index.cpp:196-209;
index.py:197-207 opens ``path + '.fmi'``), i.e. sdsl-lite's serialisation of
``csa_wt_int<>`` = ``csa_wt<wt_int<>, 32, 64, sa_order_sa_sampling<>,
isa_sampling<>, int_alphabet<>>``.

PARITY UNPINNED.  sdsl-lite is not vendored in the reference (README.md:23
clones simongog/sdsl-lite HEAD, i.e. 2.1.x; README.md:43 xxsds/sdsl-lite on
macOS), cannot be built offline, and no ``.fmi`` file exists in the reference
or this environment.  The layout below is re-derived member by member from
sdsl-lite 2.1's ``serialize()`` / ``load()`` (each field cites its class and
member) and the test writer (tests/sdsl_writer.py) restates the same
derivation, so the round trip pins the reader against the derivation, not
against a file sdsl wrote.  The reader validates everything it can from the
file itself (sizes, widths, the alphabet's C array against the decoded symbol
counts, every ISA sample against the BWT's LF walks, the SA samples against
locate), so a layout mismatch on a real sdsl file fails loudly instead of
yielding a wrong index.

Layout (little endian; ``store_to_file`` writes ``csa.serialize(out)`` with no
header):

* ``int_vector<1>`` (``bit_vector``) / ``int_vector<64>``: ``int_vector::
  write_header`` -- m_size in bits (u64) -- then ceil(m_size / 64) u64 words.
* ``int_vector<0>``: m_size in bits (u64), m_width (u8), then ceil(m_size /
  64) u64 words; element i occupies bits [i w, (i + 1) w), LSB first.
* ``rank_support_v<1>::serialize``: m_basic_block (``int_vector<64>``).
* ``select_support_mcl<b,1>::serialize``: m_arg_cnt (u64); if m_arg_cnt > 0:
  m_superblock (``int_vector<0>``), mini_or_long (``bit_vector``, empty when
  there is no long superblock), then for each of the ceil(m_arg_cnt / 4096)
  superblocks its m_longsuperblock[i] or m_miniblock[i] (``int_vector<0>``).
  Skipped: the reader needs no select.
* ``rank_support_sd`` / ``select_support_sd`` / ``*_scan``: nothing
  (``serialize_empty_object``).
* ``csa_wt::serialize``: m_wavelet_tree, m_sa_sample, m_isa_sample,
  m_alphabet -- in that order (csa_wt has no size member of its own).
* ``wt_int<>::serialize``: m_size (u64), m_sigma (u64: the number of distinct
  symbols, counted over the non-empty leaves at construction), m_tree
  (``bit_vector`` of m_size * m_max_level bits: level l at bits [l m_size,
  (l + 1) m_size), the sequence stably sorted by its top l bits, bit
  (max_level - 1 - l) of each symbol), m_tree_rank (``rank_support_v``),
  m_tree_select1 / m_tree_select0 (``select_support_mcl``), m_max_level
  (u32).  Nothing follows: m_path_off / m_path_rank_off are rebuilt by
  ``init_buffers(m_max_level)`` in ``load()`` (the zero_cnt / rank_level
  vectors belong to the wavelet matrix ``wm_int``, not to ``wt_int``).
  csa_wt constructs its wavelet tree from the cached BWT in the ORIGINAL
  alphabet (``KEY_BWT``), so the tree holds T' symbols (token id + 10 and the
  sentinel 0), not compact codes: ``interval_symbols(index.wavelet_tree, ...)``
  in fm_index.cpp:111,136 returns those symbols, which index.py:156,170 then
  filters (d > 0) and shifts back; m_max_level = hi(max symbol) + 1 (17 for a
  128k vocabulary).
* ``_sa_order_sampling`` (an ``int_vector<0>``): SA[32 i], width hi(n) + 1.
* ``_isa_sampling`` (an ``int_vector<0>``): ISA[64 k] = the row of text
  position 64 k, (n - 1) / 64 + 1 entries.
* ``int_alphabet<>`` (sdsl-lite 2.1: ``t_bit_vector = sd_vector<>``, rank /
  select ``rank_support_sd`` / ``select_support_sd``): m_char
  (``sd_vector<>::serialize``: m_size (u64), m_wl (u8), m_low (``int_vector<0>``
  of width m_wl), m_high (``bit_vector``), m_high_1_select, m_high_0_select
  (``select_support_mcl``)), m_char_rank and m_char_select (nothing), m_C
  (``int_vector<64>``, sigma + 1 cumulative counts), m_sigma (u64).  m_char is
  left default-constructed (m_size 0) when the alphabet is 0 .. sigma - 1.
  Two other alphabet encodings are accepted when the sd_vector one does not
  parse to the end of the file: ``bit_vector`` m_char with ``*_scan`` supports
  (nothing serialised) and ``bit_vector`` + ``rank_support_v`` +
  ``select_support_mcl`` (sdsl forks that changed the default).  The alphabet is
  the last member, so at most one of them consumes the file exactly and
  agrees with the decoded symbol counts; ``alphabet_layout`` says which.

Conversion: the wavelet tree is inverted on the GPU (torch, one pass per
level: ~40 bytes of device memory per row at peak) straight into the BWT of T'
(its symbols are already T' symbols), checked against the alphabet (characters
and C), handed to ``fm_initialize_from_bwt_device``; the ISA samples then give
locate / extract through ``fm_attach_isa_samples_device`` (every sample
checked by an LF walk), and the file's SA samples are compared with ``locate``
of their rows.
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
        """int_vector<1>: m_size (bits), words."""
        size = self.u64(what)
        if size > max_bits:
            raise SdslFormatError(f"{self.path}: {what} of {size} bits is implausible")
        return size, self.words(size, what)

    def int_vector0(self, what: str, max_bits: int):
        """int_vector<0>: m_size (bits), m_width (u8), words -> (count, width, words)."""
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
        """select_support_mcl<b,1>::serialize (read past it)."""
        arg_cnt = self.u64(what)
        if arg_cnt == 0:
            return
        if arg_cnt > max_bits:
            raise SdslFormatError(f"{self.path}: {what}: {arg_cnt} ones is implausible")
        sb = (arg_cnt + 4095) >> 12
        self.int_vector0(what + ".superblock", max_bits)
        mol_bits, _ = self.bit_vector(what + ".mini_or_long", max_bits)
        if mol_bits not in (0, sb):
            raise SdslFormatError(f"{self.path}: {what}: mini_or_long of {mol_bits} bits for {sb} superblocks")
        for _ in range(sb):
            self.int_vector0(what + ".block", max_bits)


def _bits_of(words: np.ndarray, nbits: int) -> np.ndarray:
    return np.unpackbits(np.ascontiguousarray(words).view(np.uint8), bitorder="little")[:nbits]


def _sd_vector_ones(c: "_Cursor", what: str, max_bits: int):
    """sd_vector<>::serialize -> (m_size, positions of its ones).  The i-th
    one at position p is stored as m_low[i] = p mod 2^wl and a set bit of
    m_high at (p >> wl) + i."""
    size = c.u64(what + ".size")
    wl = c.u8(what + ".wl")
    if size >= (1 << 40) or wl > 64:        # a logical size: sparse, so not bounded by the file
        raise SdslFormatError(f"{c.path}: {what}: size {size}, wl {wl}")
    lsize = c.u64(what + ".low")
    lw = c.u8(what + ".low")
    if lsize % max(1, lw) or lsize > max_bits or lw > 64:
        raise SdslFormatError(f"{c.path}: {what}.low: size {lsize} bits, width {lw}")
    lwords = c.words(lsize, what + ".low")
    cnt = lsize // lw if lw else 0
    hbits, hwords = c.bit_vector(what + ".high", max_bits)
    c.skip_select_mcl(what + ".high_1_select", max_bits)
    c.skip_select_mcl(what + ".high_0_select", max_bits)
    if size == 0:
        if cnt:
            raise SdslFormatError(f"{c.path}: {what}: empty vector with {cnt} ones")
        return 0, np.zeros(0, dtype=np.int64)
    if lw != wl:
        raise SdslFormatError(f"{c.path}: {what}: low width {lw} != wl {wl}")
    hpos = np.flatnonzero(_bits_of(hwords, hbits)).astype(np.int64)
    if hpos.size != cnt:
        raise SdslFormatError(f"{c.path}: {what}: {hpos.size} high bits for {cnt} ones")
    low = unpack_int_vector(lwords, cnt, wl).astype(np.int64) if wl else np.zeros(cnt, dtype=np.int64)
    pos = ((hpos - np.arange(cnt, dtype=np.int64)) << wl) | low
    if cnt and (np.any(np.diff(pos) <= 0) or pos[-1] >= size):
        raise SdslFormatError(f"{c.path}: {what}: ones not strictly increasing inside {size} bits")
    return size, pos


def _read_alphabet(c: "_Cursor", layout: str, cap: int):
    """int_alphabet<...>::serialize in one of the accepted encodings ->
    (chars or None for the identity, C, sigma)."""
    if layout == "sd_vector":
        size, chars = _sd_vector_ones(c, "alphabet.char", cap)
        chars = chars if size else None
    else:
        nbits, words = c.bit_vector("alphabet.char", cap)
        chars = np.flatnonzero(_bits_of(words, nbits)).astype(np.int64) if nbits else None
        if layout == "bit_vector+v+mcl":
            c.int_vector64("alphabet.char_rank", cap)
            c.skip_select_mcl("alphabet.char_select", cap)
    C = c.int_vector64("alphabet.C", cap).copy()
    sigma = c.u64("alphabet.sigma")
    return chars, C, sigma


ALPHABET_LAYOUTS = ("sd_vector", "bit_vector+scan", "bit_vector+v+mcl")


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
        # ---- csa_wt::m_wavelet_tree (wt_int<>::serialize)
        self.n = c.u64("wt_int.m_size")
        self.wt_sigma = c.u64("wt_int.m_sigma")
        if self.n == 0 or self.n >= (1 << 34):
            raise SdslFormatError(f"{path}: wt_int size {self.n} out of range (0 < n < 2^34)")
        tree_bits, self.tree = c.bit_vector("wt_int.m_tree", cap)
        c.int_vector64("wt_int.m_tree_rank", cap)
        c.skip_select_mcl("wt_int.m_tree_select1", cap)
        c.skip_select_mcl("wt_int.m_tree_select0", cap)
        self.max_level = c.u32("wt_int.m_max_level")
        if not 1 <= self.max_level <= 64 or self.max_level * self.n != tree_bits:
            raise SdslFormatError(f"{path}: wt_int m_max_level {self.max_level} does not match a tree of "
                                  f"{tree_bits} bits over {self.n} rows")
        # ---- csa_wt::m_sa_sample, m_isa_sample
        cnt, width, words = c.int_vector0("sa_samples", cap)
        if cnt != (self.n + SDSL_SA_RATE - 1) // SDSL_SA_RATE:
            raise SdslFormatError(f"{path}: {cnt} SA samples for n = {self.n}")
        self.sa_samples = unpack_int_vector(words, cnt, width)
        cnt, width, words = c.int_vector0("isa_samples", cap)
        if cnt != (self.n - 1) // SDSL_ISA_RATE + 1:
            raise SdslFormatError(f"{path}: {cnt} ISA samples for n = {self.n}")
        self.isa_samples = unpack_int_vector(words, cnt, width)
        # ---- csa_wt::m_alphabet: the first encoding that ends exactly at the end of the file
        start, errors = c.p, []
        for layout in ALPHABET_LAYOUTS:
            c.p = start
            try:
                chars, C, sigma = _read_alphabet(c, layout, cap)
            except SdslFormatError as e:
                errors.append(f"{layout}: {e}")
                continue
            if c.p != buf.size:
                errors.append(f"{layout}: {buf.size - c.p} trailing bytes")
                continue
            if C.size != sigma + 1 or int(C[-1]) != self.n or np.any(np.diff(C.astype(np.int64)) < 0):
                errors.append(f"{layout}: C array inconsistent with sigma {sigma} / n {self.n}")
                continue
            if chars is not None and chars.size != sigma:
                errors.append(f"{layout}: {chars.size} characters for sigma {sigma}")
                continue
            self.alphabet_layout = layout
            self.C, self.sigma = C, sigma
            self.chars = chars if chars is not None else np.arange(sigma, dtype=np.int64)
            break
        else:
            raise SdslFormatError(f"{path}: the alphabet does not parse in any accepted encoding: " +
                                  "; ".join(errors))
        # m_sigma counts the distinct symbols of the tree (= the alphabet's sigma)
        if self.wt_sigma != self.sigma:
            raise SdslFormatError(f"{path}: wavelet tree sigma {self.wt_sigma} != alphabet sigma {self.sigma}")
        if self.sigma and self.max_level < max(1, int(self.chars[-1]).bit_length()):
            raise SdslFormatError(f"{path}: {self.max_level} levels cannot hold symbol {int(self.chars[-1])}")

    @property
    def comp2char(self) -> np.ndarray:
        """Compact code -> character (the alphabet's characters, ascending)."""
        return self.chars


def decode_wt_int_device(tree_words: np.ndarray, n: int, L: int, device, chunk: int = 1 << 27):
    """The sequence a wt_int tree encodes (int64 [n] on ``device``; for a
    csa_wt_int<> these are the BWT's T' symbols), by one pass per level: every position carries its prefix
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


def load_sdsl_fmi(path: str, device: Optional[int] = None, verify_samples: bool = True, options=None):
    """An engine FMIndex (fmidx.fm_index.FMIndex, the SWIG surface) from a
    reference ``.fmi`` file (see the module docstring; parity unpinned)."""
    import torch

    from ._lib import check, lib
    from .fm_index import FMIndex, _default_device, _stream_of
    from ctypes import c_void_p

    f = SdslCsaWtInt(path)
    dev_index = _default_device() if device is None else int(device)
    dev = torch.device("cuda", dev_index)
    sym = decode_wt_int_device(f.tree, f.n, f.max_level, dev)     # T' symbols (csa_wt builds from KEY_BWT)
    counts = torch.bincount(sym, minlength=int(f.chars[-1]) + 1 if f.sigma else 1).cpu().numpy()
    want = np.zeros(counts.size, dtype=np.int64)
    if counts.size != (int(f.chars[-1]) + 1 if f.sigma else 1):
        raise SdslFormatError(f"{path}: the wavelet tree holds symbols beyond the alphabet")
    want[f.chars] = np.diff(f.C.astype(np.int64))
    if not np.array_equal(counts.astype(np.int64), want):
        raise SdslFormatError(f"{path}: decoded wavelet tree disagrees with the alphabet's characters / C array")
    bwt = sym.to(torch.int32)
    del sym
    if int((bwt == 0).sum()) != 1:
        raise SdslFormatError(f"{path}: the decoded BWT must hold exactly one sentinel 0")
    ix = FMIndex(device=dev_index, options=options)
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


__all__ = ["ALPHABET_LAYOUTS", "SdslCsaWtInt", "SdslFormatError", "decode_wt_int_device", "load_sdsl_fmi", "is_sdsl_file",
           "unpack_int_vector"]
