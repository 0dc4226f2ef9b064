"""The builder CLI (fmidx/build_index.py) against the reference's
build_fm_index.py semantics: passage parsing and cleaning
(build_fm_index.py:52-97), the streaming T' encoder against index.py:47-53,
and (GPU) the device-built index equal to FMIndex.initialize on the same
sequences, through save/load."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]

from fmidx.build_index import CorpusBuffer, build_index, preprocess_file  # noqa: E402
from fmidx.index import encode_corpus  # noqa: E402

KILT = ("p1\tAthena\tAthena   or  Athene,\tis a goddess.\n"     # text keeps its own tab
        "p2\tShort\n"                                          # 2 fields: skipped
        "p3\tBullets\tBULLET::::one SECTION::::two\n"
        "p4\tEmpty\t   \n"                                     # empty text: skipped, no label
        "p5\tMixed\tUPPER lower\n")
DPR = ("id\ttext\ttitle\n"
       "10\t\"quoted text, with tab\tinside\"\tT1\n"
       "11\tplain text\tT2\n"
       "12\tonly two\n")


def _write(tmp_path, name, s):
    p = tmp_path / name
    p.write_text(s)
    return str(p)


def test_preprocess_kilt(tmp_path):
    path = _write(tmp_path, "k.tsv", KILT)
    labels = []
    out = list(preprocess_file(path, labels, "kilt"))
    assert out == ["Athena or Athene, is a goddess.", "one two", "UPPER lower"]
    assert labels == ["p1", "p3", "p5"]
    labels = []
    out = list(preprocess_file(path, labels, "kilt", include_title=True, lowercase=True, delim="@@"))
    assert out == ["athena @@ athena or athene, is a goddess.", "bullets @@ one two", "mixed @@ upper lower"]


def test_preprocess_dpr(tmp_path):
    path = _write(tmp_path, "d.tsv", DPR)
    labels = []
    out = list(preprocess_file(path, labels, "dpr", include_title=True, delim="|"))
    assert out == ["T1 | quoted text, with tab inside", "T2 | plain text"]
    assert labels == ["10", "11"]


def test_clean_passage_edges(tmp_path):
    from fmidx.build_index import PassageRules, clean_passage

    # an empty title still contributes "<title> <delim> " (build_fm_index.py:87-90)
    assert clean_passage("  ", "x\n y", PassageRules(include_title=True)) == " @@ x y"
    assert clean_passage("T", "BULLET:::: SECTION::::", PassageRules(include_title=True)) is None
    split = PassageRules(include_title=True, delim="|", word_tokenize=lambda s: s.replace(",", " , ").split())
    assert clean_passage("A,B", "c,d  e", split) == "A , B | c , d e"
    # --tokenize without a word tokenizer is refused before the file is read
    with pytest.raises(RuntimeError):
        list(preprocess_file(str(tmp_path / "absent.tsv"), [], "kilt", tokenize=True))
    with pytest.raises(ValueError):
        list(preprocess_file(_write(tmp_path, "x.tsv", KILT), [], "csv"))


def test_encode_passage_prompt():
    from fmidx.build_index import encode_passage

    class Tok:                                   # records the prompt; ids = its bytes
        eos_token_id = 2
        seen = []

        def __call__(self, text, add_special_tokens):
            assert add_special_tokens is False
            self.seen.append(text)
            return {"input_ids": list(text.encode())}

    tok = Tok()
    assert encode_passage(tok, "  hi ") == list(b"Paraphrase: hi") + [2]
    assert encode_passage(tok, "hi", bart=True) == list(b"Paraphrase:  hi") + [2]


def test_corpus_buffer_matches_encoding():
    rng = np.random.default_rng(3)
    docs = [rng.integers(-9, 300000, size=int(rng.integers(0, 50))).tolist() for _ in range(300)]
    cb = CorpusBuffer(capacity=16)
    for d in docs:
        cb.append(d)
    data, beginnings, occurring = encode_corpus(docs)
    t = cb.text()
    assert t[-1] == 0 and np.array_equal(t[:-1].astype(np.uint64), data)
    assert cb.beginnings == beginnings
    assert cb.occurring == occurring
    with pytest.raises(OverflowError):
        CorpusBuffer().append([5, -10])


@pytest.mark.gpu
def test_build_index_on_device_equals_initialize(tmp_path):
    from fmidx.build_index import index_from_sequences
    from fmidx.index import FMIndex

    rng = np.random.default_rng(8)
    docs = [rng.integers(0, 50, size=int(rng.integers(1, 60))).tolist() for _ in range(400)]
    a = index_from_sequences(docs, device=0)
    b = FMIndex(device=0)
    b.initialize(docs)
    assert a.size() == b.size() and a.beginnings == b.beginnings
    assert sorted(a.occurring) == sorted(b.occurring)
    assert a.occurring_distinct == b.occurring_distinct and a.occurring_counts == b.occurring_counts
    pats = [d[i:i + k] for d in docs[:60] for i, k in [(0, 1), (1, 3), (2, 5)]] + [[99], [], [7, 7, 7, 7]]
    assert a.get_ranges(pats) == b.get_ranges(pats)
    lows = [lo for lo, _ in b.get_ranges(pats)]
    highs = [hi for _, hi in b.get_ranges(pats)]
    assert a.get_distinct_count_multi(lows, highs) == b.get_distinct_count_multi(lows, highs)
    assert [a.get_doc(i) for i in range(0, 400, 37)] == [b.get_doc(i) for i in range(0, 400, 37)]
    # the CLI path: parse a KILT file, byte-level tokens, save, load
    path = _write(tmp_path, "k.tsv", KILT)
    ix = build_index(path, encode=lambda s: list(s.encode()), include_title=True, device=0)
    assert ix.labels == ["p1", "p3", "p5"] and ix.n_docs == 3
    seqs = [list(t.encode()) for t in preprocess_file(path, [], "kilt", include_title=True)]
    ref = FMIndex(device=0)
    ref.initialize(seqs)
    assert [ix.get_doc(i) for i in range(3)] == [ref.get_doc(i) for i in range(3)]
    assert ix.occurring_distinct == ref.occurring_distinct
    out = str(tmp_path / "idx")
    ix.save(out)
    back = FMIndex.load(out, device=0)
    assert back.labels == ix.labels and back.beginnings == ix.beginnings
    assert back.get_ranges([list(b"goddess"), list(b"two")]) == ix.get_ranges([list(b"goddess"), list(b"two")])
    assert back.get_count(list(b"goddess")) == 1
