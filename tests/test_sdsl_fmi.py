"""The reader of the reference's ``.fmi`` (sdsl csa_wt_int<> serialisation,
fm_index.cpp:196-209, index.py:197-207) -- PARITY UNPINNED: there is no sdsl
build and no .fmi file here, so the reader is checked against
tests/sdsl_writer.py, a restatement of the same layout, plus the reader's own
consistency checks (C array vs decoded counts, ISA walks, SA samples).

CPU: parsing and the wavelet-tree inversion (on torch's CPU device).
GPU: a reference-layout file loaded through FMIndex.load == the oracle on every
query surface; corrupt files refused."""
import pickle

import numpy as np
import pytest

from oracle.fm_oracle import OracleIndex, encode_corpus
from tests.sdsl_writer import write_csa_wt_int


def _docs(seed, n_docs, vocab, max_len):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, vocab, size=int(rng.integers(1, max_len + 1))).tolist() for _ in range(n_docs)]


def _text(docs):
    enc = encode_corpus(docs)
    text = enc[0] if isinstance(enc, tuple) else enc
    return np.concatenate([np.asarray(text, dtype=np.int64), [0]])


CASES = [(1, 3, 5, 4), (2, 40, 30, 60), (3, 200, 500, 120), (4, 30, 128256, 80), (5, 1, 2, 63)]


@pytest.mark.parametrize("seed,n_docs,vocab,max_len", CASES)
@pytest.mark.parametrize("layout", ["sd_vector", "bit_vector+scan", "bit_vector+v+mcl"])
def test_parse_and_invert_on_cpu(tmp_path, seed, n_docs, vocab, max_len, layout):
    import torch

    from fmidx.sdsl_fmi import SdslCsaWtInt, decode_wt_int_device

    text = _text(_docs(seed, n_docs, vocab, max_len))
    p = str(tmp_path / "x.fmi")
    ref = write_csa_wt_int(p, text, alphabet_layout=layout)
    f = SdslCsaWtInt(p)
    n = text.size
    assert f.n == n and f.max_level == ref["L"] and f.sigma == ref["sigma"]
    assert f.alphabet_layout == layout
    assert np.array_equal(f.chars, np.unique(text))
    assert np.array_equal(f.sa_samples.astype(np.int64), ref["sa"][::32])
    isa = np.empty(n, dtype=np.int64)
    isa[ref["sa"]] = np.arange(n)
    assert np.array_equal(f.isa_samples.astype(np.int64), isa[::64])
    # the tree holds the BWT's T' symbols themselves (csa_wt builds it from KEY_BWT)
    sym = decode_wt_int_device(f.tree, n, f.max_level, torch.device("cpu"), chunk=1000)
    assert np.array_equal(sym.numpy(), ref["bwt"])


def _hand_fmi_bytes() -> bytes:
    """csa_wt_int<> of T' = [11, 12, 11, 0] assembled field by field by hand
    (independent of tests/sdsl_writer.py): SA = [3, 2, 0, 1], BWT = [11, 12,
    0, 11], 4 levels (hi(12) + 1); level bits 1101 | 0010 | 0110 | 0110 (level
    l+1 in the stable order of the top l+1 bits) = word 0x664B; alphabet {0,
    11, 12} as an sd_vector of 13 bits (wl = 4 - 2 = 2: low [0, 3, 0], high
    bits 0, 3, 5 of 7), C = [0, 1, 3, 4]."""
    import struct

    q = lambda v: struct.pack("<Q", v)      # noqa: E731
    b = lambda v: struct.pack("<B", v)      # noqa: E731
    i32 = lambda v: struct.pack("<I", v)    # noqa: E731
    rank_word = sum(8 << (9 * j) for j in range(7))      # 8 ones in word 0: every in-block prefix is 8
    mcl = lambda: q(8) + q(5) + b(5) + q(0) + q(0) + q(1) + b(1) + q(0)   # noqa: E731 -- 8 ones / 8 zeros
    out = b"".join([
        q(4), q(3),                                  # wt_int m_size, m_sigma
        q(16), q(0x664B),                            # m_tree
        q(128), q(0), q(rank_word),                  # m_tree_rank: m_basic_block
        mcl(), mcl(),                                # m_tree_select1 / 0: superblock [0] w5, no mini_or_long, [0] w1
        i32(4),                                      # m_max_level
        q(3), b(3), q(3),                            # sa samples: [3]
        q(3), b(3), q(2),                            # isa samples: [2]
        q(13), b(2), q(6), b(2), q(0 | 3 << 2),      # m_char sd_vector: size, wl, m_low [0, 3, 0]
        q(7), q(1 | 8 | 32),                         # m_high
        q(3), q(3), b(1), q(0), q(0), q(1), b(1), q(0),   # high_1_select (3 ones at 0, 3, 5)
        q(4), q(3), b(1), q(1), q(0), q(1), b(1), q(0),   # high_0_select (4 zeros from 1)
        q(256), q(0), q(1), q(3), q(4),              # m_C
        q(3),                                        # m_sigma
    ])
    return out


def test_hand_assembled_fmi(tmp_path):
    """A four-row file written byte by byte from the derivation: the reader
    recovers n, the levels, the samples, the alphabet and the BWT; the test
    writer produces the same bytes except the select structures it is free to
    shape (the reader skips them)."""
    import torch

    from fmidx.sdsl_fmi import SdslCsaWtInt, decode_wt_int_device

    p = str(tmp_path / "hand.fmi")
    open(p, "wb").write(_hand_fmi_bytes())
    f = SdslCsaWtInt(p)
    assert (f.n, f.wt_sigma, f.max_level, f.sigma, f.alphabet_layout) == (4, 3, 4, 3, "sd_vector")
    assert f.chars.tolist() == [0, 11, 12] and f.C.tolist() == [0, 1, 3, 4]
    assert f.sa_samples.tolist() == [3] and f.isa_samples.tolist() == [2]
    assert decode_wt_int_device(f.tree, 4, 4, torch.device("cpu")).tolist() == [11, 12, 0, 11]
    w = str(tmp_path / "writer.fmi")
    ref = write_csa_wt_int(w, np.array([11, 12, 11, 0]))
    assert ref["sa"].tolist() == [3, 2, 0, 1] and ref["bwt"].tolist() == [11, 12, 0, 11]
    g = SdslCsaWtInt(w)
    assert g.tree.tolist() == f.tree.tolist() and g.chars.tolist() == f.chars.tolist()


def test_wavelet_matrix_trailer_is_refused(tmp_path):
    """wm_int's zero_cnt / rank_level after m_max_level (what round 3's reader
    expected) are not part of wt_int: such a file does not parse."""
    from fmidx.sdsl_fmi import SdslCsaWtInt, SdslFormatError

    good = _hand_fmi_bytes()
    cut = 8 + 8 + 16 + 24 + 2 * 53 + 4          # through m_max_level
    trailer = (256).to_bytes(8, "little") + bytes(32) + (256).to_bytes(8, "little") + bytes(32)
    p = str(tmp_path / "wm.fmi")
    open(p, "wb").write(good[:cut] + trailer + good[cut:])
    with pytest.raises(SdslFormatError):
        SdslCsaWtInt(p)


def test_contiguous_alphabet_and_corrupt_files(tmp_path):
    from fmidx.sdsl_fmi import SdslCsaWtInt, SdslFormatError

    text = np.array([1, 2, 3, 1, 2, 4, 2, 3, 1, 0], dtype=np.int64)      # chars 0..4: contiguous
    p = str(tmp_path / "c.fmi")
    write_csa_wt_int(p, text)
    f = SdslCsaWtInt(p)
    assert np.array_equal(f.comp2char, np.arange(5)) and f.alphabet_layout == "sd_vector"
    good = open(p, "rb").read()
    for name, bad in [("truncated", good[:-1]), ("trailing", good + b"\0"), ("header only", good[:16]),
                      ("empty", b""), ("n = 0", b"\0" * 8 + good[8:]),
                      ("n huge", (1 << 40).to_bytes(8, "little") + good[8:])]:
        q = str(tmp_path / "bad.fmi")
        open(q, "wb").write(bad)
        with pytest.raises(SdslFormatError):
            SdslCsaWtInt(q)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n_docs,vocab,max_len", CASES[1:] + [(6, 2000, 3000, 300)])
def test_reference_fmi_loads_and_answers_like_the_oracle(tmp_path, seed, n_docs, vocab, max_len):
    """index.FMIndex.load(path) with a reference-layout path.fmi and the
    reference's pickled path.oth: every query surface == the oracle."""
    from fmidx.index import FMIndex

    docs = _docs(seed, n_docs, vocab, max_len)
    ora = OracleIndex()
    ora.initialize(docs, in_memory=True)
    text = _text(docs)
    assert np.array_equal(text, np.asarray(ora.text, dtype=np.int64))
    base = str(tmp_path / "idx")
    write_csa_wt_int(base + ".fmi", text)
    with open(base + ".oth", "wb") as fh:          # index.py:194's pickle
        pickle.dump((list(ora.beginnings), list(ora.occurring), None), fh)
    ix = FMIndex.load(base, device=0)
    n = ora.size()
    assert ix.size() == n and ix.beginnings == ora.beginnings
    assert ix.occurring_distinct == ora.occurring_distinct
    rng = np.random.default_rng(seed)
    F = [t for d in reversed(docs) for t in d]
    pats = [F[s:s + int(rng.integers(1, 6))] for s in rng.integers(0, len(F), size=200)] + [[vocab + 3], []]
    assert ix.get_ranges(pats) == [ora.get_range(p) for p in pats]
    for _ in range(60):
        a = int(rng.integers(0, n))
        b = int(rng.integers(a, n + 1))
        assert ix.distinct_count(a, b) == ora.distinct_count(a, b)
    for r in list(range(min(n, 300))) + [n - 1, n]:
        assert ix.locate(r) == ora.locate(r)
    for d in range(min(len(docs), 40)):
        assert ix.get_doc(d) == ora.get_doc(d)
    a = int(rng.integers(0, n - 1))
    assert ix.extract_text(a, n) == ora.extract_text(a, n)


@pytest.mark.gpu
def test_corrupt_reference_fmi_is_refused(tmp_path):
    """A flipped wavelet-tree bit (the decoded counts no longer match C, or the
    ISA walks miss their samples) and a corrupted ISA sample are refused with
    an error -- the engine never answers from an inconsistent index."""
    from fmidx import FMIndexError
    from fmidx.fm_index import load_FMIndex
    from fmidx.sdsl_fmi import SdslCsaWtInt, SdslFormatError

    text = _text(_docs(9, 300, 400, 100))
    p = str(tmp_path / "g.fmi")
    write_csa_wt_int(p, text)
    ok = load_FMIndex(p, device=0)
    assert ok.size() == text.size
    good = bytearray(open(p, "rb").read())
    # the tree's first data word starts after size (8), sigma (8), tree size (8)
    bad = bytearray(good)
    bad[24 + 5] ^= 0x10
    q = str(tmp_path / "b.fmi")
    open(q, "wb").write(bytes(bad))
    with pytest.raises((SdslFormatError, FMIndexError)):
        load_FMIndex(q, device=0)
    # an ISA sample moved to another row: locate must not be built from it
    f = SdslCsaWtInt(p)
    raw = open(p, "rb").read()
    isa_words = f.isa_samples
    k = 3
    width = max(1, int(text.size).bit_length())
    # locate the isa int_vector: the SA samples vector precedes it; find it by its header
    hdr = (isa_words.size * width).to_bytes(8, "little") + bytes([width])
    at = raw.rfind(hdr)
    assert at > 0
    data = bytearray(raw)
    bit = (at + 9) * 8 + k * width
    cur = int(isa_words[k])
    new = cur ^ 1
    for j in range(width):
        byte, off = divmod(bit + j, 8)
        if (new >> j) & 1:
            data[byte] |= 1 << off
        else:
            data[byte] &= ~(1 << off) & 0xFF
    open(q, "wb").write(bytes(data))
    with pytest.raises((SdslFormatError, FMIndexError)):
        load_FMIndex(q, device=0)
