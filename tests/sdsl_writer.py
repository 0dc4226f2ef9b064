"""TEST INFRASTRUCTURE: a writer of sdsl-lite's csa_wt_int<> serialisation (the
reference's ``.fmi``, fm_index.cpp:196-199) for the reader's round-trip tests.

It is restated from sdsl-lite 2.1's ``serialize()`` member order, member by
member (the class and member of every field are named below and in
fmidx/sdsl_fmi.py's header), from a text T' by definition (suffix array by
sorting, oracle/fm_oracle.py):

* csa_wt: m_wavelet_tree, m_sa_sample, m_isa_sample, m_alphabet.
* wt_int<>: m_size, m_sigma (distinct symbols), m_tree (levels of the
  ORIGINAL BWT symbols -- csa_wt builds its tree from KEY_BWT), m_tree_rank
  (rank_support_v), m_tree_select1, m_tree_select0 (select_support_mcl),
  m_max_level (u32) -- and nothing after it.
* int_alphabet<> with sd_vector<> m_char (m_size, m_wl, m_low, m_high,
  m_high_1_select, m_high_0_select; sdsl's sd_vector(bit_vector) choice of
  wl), rank_support_sd / select_support_sd (empty), m_C (int_vector<64>),
  m_sigma.  ``alphabet_layout`` writes the two other encodings the reader
  accepts.

The rank directories are computed as sdsl's rank_support_v lays them out;
the select structures (which the reader skips) are written in sdsl's shape --
arg_cnt, a superblock vector, an empty mini_or_long, one miniblock vector per
4096 ones -- without claiming sdsl's exact long/mini choice.  No sdsl file
exists here, so this pins the reader against this restatement only (parity
unpinned, as the reader's header says).
"""
from __future__ import annotations

import io
import struct

import numpy as np

from oracle.fm_oracle import suffix_array


def _bits_needed(x: int) -> int:
    return max(1, int(x).bit_length())


def _words(bits: np.ndarray) -> np.ndarray:
    nw = (bits.size + 63) // 64
    buf = np.zeros(nw * 64, dtype=np.uint8)
    buf[: bits.size] = bits
    return np.packbits(buf, bitorder="little").view(np.uint64) if nw else np.zeros(0, dtype=np.uint64)


class _W:
    def __init__(self):
        self.f = io.BytesIO()

    def u64(self, v):
        self.f.write(struct.pack("<Q", int(v)))

    def u32(self, v):
        self.f.write(struct.pack("<I", int(v)))

    def u8(self, v):
        self.f.write(struct.pack("<B", int(v)))

    def raw(self, words: np.ndarray):
        self.f.write(np.ascontiguousarray(words, dtype=np.uint64).tobytes())

    def bit_vector(self, bits: np.ndarray):
        self.u64(bits.size)
        self.raw(_words(bits.astype(np.uint8)))

    def int_vector64(self, vals):
        vals = np.asarray(vals, dtype=np.uint64)
        self.u64(64 * vals.size)
        self.raw(vals)

    def int_vector0(self, vals, width: int):
        vals = np.asarray(vals, dtype=np.uint64)
        self.u64(vals.size * width)
        self.u8(width)
        bits = ((vals[:, None] >> np.arange(width, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(np.uint8)
        self.raw(_words(bits.reshape(-1)))

    def rank_support_v(self, bits: np.ndarray):
        """sdsl rank_support_v<1>: per 512-bit block the ones before it and the
        7 in-block 9-bit prefix counts of words 1..7; one extra pair at the end."""
        words = _words(bits.astype(np.uint8))
        nblk = (words.size * 64 >> 9) + 1
        pop = np.array([bin(int(w)).count("1") for w in words], dtype=np.uint64)
        pop = np.concatenate([pop, np.zeros(nblk * 8 - pop.size, dtype=np.uint64)])
        per = pop.reshape(nblk, 8)
        before = np.concatenate([[0], np.cumsum(per.sum(1))[:-1]]).astype(np.uint64)
        inner = np.cumsum(per, 1)
        packed = np.zeros(nblk, dtype=np.uint64)
        for j in range(1, 8):
            packed |= inner[:, j - 1] << np.uint64(9 * (j - 1))
        d = np.empty(2 * nblk, dtype=np.uint64)
        d[0::2] = before
        d[1::2] = packed
        self.int_vector64(d)

    def select_support_mcl(self, bits: np.ndarray, one: bool):
        pos = np.flatnonzero(bits == (1 if one else 0)).astype(np.uint64)
        self.u64(pos.size)
        if pos.size == 0:
            return
        n = max(1, bits.size)
        sb = (pos.size + 4095) // 4096
        self.int_vector0(pos[::4096][:sb], _bits_needed(n))
        self.bit_vector(np.zeros(0, dtype=np.uint8))            # mini_or_long: no long superblocks
        for i in range(sb):
            blk = pos[4096 * i: 4096 * (i + 1)]
            rel = (blk[::64] - blk[0]).astype(np.uint64)
            self.int_vector0(rel, _bits_needed(int(rel.max()) if rel.size else 1))


def wt_int_tree(seq: np.ndarray, L: int) -> np.ndarray:
    """The concatenated level bits of sdsl's wt_int over ``seq``."""
    n = seq.size
    out = np.zeros(n * L, dtype=np.uint8)
    s = seq.astype(np.int64)
    for lev in range(L):
        cur = s if lev == 0 else s[np.argsort(s >> (L - lev), kind="stable")]
        out[lev * n:(lev + 1) * n] = (cur >> (L - 1 - lev)) & 1
    return out


def _hi(x: int) -> int:
    """sdsl bits::hi: index of the most significant set bit (-1 for 0)."""
    return int(x).bit_length() - 1


def sd_vector(w: "_W", bits: np.ndarray):
    """sd_vector<>::serialize of the bit_vector ``bits`` (sd_vector(const
    bit_vector&): logm = hi(m) + 1, logn = hi(size) + 1, logm decremented when
    equal, wl = logn - logm; m_low[i] = p & (2^wl - 1); m_high[(p >> wl) + i]
    set; m_high of m + 2^logm bits)."""
    size = bits.size
    ones = np.flatnonzero(bits).astype(np.int64)
    m = ones.size
    if size == 0:                              # default-constructed: the continuous alphabet
        w.u64(0)
        w.u8(0)
        w.int_vector0(np.zeros(0, dtype=np.uint64), 64)
        w.bit_vector(np.zeros(0, dtype=np.uint8))
        w.select_support_mcl(np.zeros(0, dtype=np.uint8), True)
        w.select_support_mcl(np.zeros(0, dtype=np.uint8), False)
        return
    logm = _hi(m) + 1
    logn = _hi(size) + 1
    if logm == logn:
        logm -= 1
    wl = logn - logm
    high = np.zeros(m + (1 << logm), dtype=np.uint8)
    high[(ones >> wl) + np.arange(m)] = 1
    w.u64(size)
    w.u8(wl)
    w.int_vector0(ones & ((1 << wl) - 1), wl)
    w.bit_vector(high)
    w.select_support_mcl(high, True)
    w.select_support_mcl(high, False)


def write_csa_wt_int(path: str, text: np.ndarray, contiguous_alphabet=None, alphabet_layout: str = "sd_vector"):
    """Serialise the csa_wt_int<> of T' (``text``: int array, unique 0 last)."""
    text = np.asarray(text, dtype=np.int64)
    n = text.size
    sa = suffix_array(text).astype(np.int64)
    bwt = text[(sa + n - 1) % n]
    chars = np.unique(text)
    contiguous = bool(chars.size == chars[-1] + 1) if contiguous_alphabet is None else contiguous_alphabet
    sigma = chars.size
    # wt_int over the original BWT symbols: m_max_level = hi(max(1, max symbol)) + 1
    L = _hi(max(1, int(bwt.max()))) + 1
    tree = wt_int_tree(bwt, L)
    w = _W()
    # csa_wt::m_wavelet_tree = wt_int<>::serialize
    w.u64(n)                      # m_size
    w.u64(sigma)                  # m_sigma: distinct symbols (non-empty leaves)
    w.bit_vector(tree)            # m_tree
    w.rank_support_v(tree)        # m_tree_rank
    w.select_support_mcl(tree, True)    # m_tree_select1
    w.select_support_mcl(tree, False)   # m_tree_select0
    w.u32(L)                      # m_max_level (uint32_t); m_path_off / m_path_rank_off are not stored
    # csa_wt::m_sa_sample (_sa_order_sampling = int_vector<0>, width hi(n) + 1), m_isa_sample
    wid = _hi(n) + 1
    w.int_vector0(sa[::32], wid)
    isa = np.empty(n, dtype=np.int64)
    isa[sa] = np.arange(n)
    w.int_vector0(isa[::64], wid)
    # csa_wt::m_alphabet = int_alphabet<>::serialize
    cb = np.zeros(0 if contiguous else int(chars[-1]) + 1, dtype=np.uint8)
    cb[chars[chars < cb.size]] = 1
    if alphabet_layout == "sd_vector":
        sd_vector(w, cb)          # m_char; m_char_rank (rank_support_sd), m_char_select: nothing
    elif alphabet_layout == "bit_vector+scan":
        w.bit_vector(cb)          # m_char; rank_support_scan / select_support_scan: nothing
    elif alphabet_layout == "bit_vector+v+mcl":
        w.bit_vector(cb)
        w.rank_support_v(cb)
        w.select_support_mcl(cb, True)
    else:
        raise ValueError(alphabet_layout)
    C = np.concatenate([[0], np.cumsum(np.bincount(np.searchsorted(chars, bwt), minlength=sigma))]).astype(np.uint64)
    w.int_vector64(C)             # m_C
    w.u64(sigma)                  # m_sigma
    with open(path, "wb") as f:
        f.write(w.f.getvalue())
    return {"n": n, "sa": sa, "bwt": bwt, "L": L, "sigma": sigma, "chars": chars}
