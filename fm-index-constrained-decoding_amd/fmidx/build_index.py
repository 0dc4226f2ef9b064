"""Index construction from a passage file -- the reference's builder CLI
(build_fm_index.py:1-156) on the MI355X engine.

Same inputs, arguments and output: a KILT (``id<TAB>title<TAB>text``) or DPR
(header line, then ``id<TAB>text<TAB>title`` csv) file; each passage cleaned
as in ``preprocess_file`` (build_fm_index.py:52-97: whitespace runs -> one
space, ``ftfy.fix_text``, the ``BULLET::::`` / ``SECTION::::`` markers
dropped, empty texts skipped, optional ``"{title} {delim} "`` prefix and
lowercasing, the passage id appended to ``labels``), tokenized as in
``process`` (build_fm_index.py:37-50: ``"Paraphrase: " + text`` with no
special tokens, then eos; a leading space for BART models) by a pool of
workers, and saved as ``<output>.fmi`` + ``<output>.oth``.

What differs is how the corpus reaches the index.  The reference collects
every token sequence in host memory and runs sdsl's host suffix sorting
(``FMIndex.initialize`` -> ``construct_im``), which does not fit an
enwiki-scale corpus in host RAM.  Here the token stream is
encoded as it arrives into one growing uint32 buffer of T' symbols (each doc
reversed, ids + SHIFT, exactly index.py:47-53), uploaded once, and the whole
index -- suffix array, BWT, every query structure -- is built on the GPU
(``fm_initialize_from_text_device``).

Offline notes: ``ftfy`` is used when importable (it is not in this image; the
text is then left as is, which changes nothing for ASCII input);
``--hf_model`` must name a tokenizer available locally (no downloads); the
reference's default, fairseq BART via ``torch.hub``, needs the network and is
refused with a clear error.
"""
from __future__ import annotations

import argparse
import contextlib
import csv
import multiprocessing
import re
from dataclasses import dataclass
from functools import partial
from typing import Callable, Iterable, Iterator, List, Optional, Sequence, Tuple

import numpy as np

from .index import SHIFT, FMIndex

try:                                    # build_fm_index.py:13
    from ftfy import fix_text as _fix_text
except ImportError:                     # pragma: no cover - not in this image
    def _fix_text(text: str) -> str:
        return text


_WHITESPACE = re.compile(r"\s+")
_WIKI_MARKERS = ("BULLET::::", "SECTION::::")


@dataclass(frozen=True)
class PassageRules:
    """How a passage becomes index text (build_fm_index.py:69-95 and its
    ``--include_title / --delim / --lowercase / --tokenize`` flags)."""
    include_title: bool = False
    delim: str = "@@"
    lowercase: bool = False
    word_tokenize: Optional[Callable[[str], List[str]]] = None


def read_records(f, format: str) -> Iterator[Tuple[str, str, str]]:
    """(id, title, text) for every well-formed record of an open passage file:
    KILT lines ``id<TAB>title<TAB>text`` (build_fm_index.py:61-65), DPR csv
    rows ``id<TAB>text<TAB>title`` after one header line (:55-59); records
    without exactly three fields are skipped, as there."""
    if format == "kilt":
        for line in f:
            fields = line.strip().split("\t", 2)
            if len(fields) == 3:
                yield fields[0], fields[1], fields[2]
    elif format == "dpr":
        next(f, None)
        for fields in csv.reader(f, delimiter="\t", quotechar='"'):
            if len(fields) == 3:
                pid, text, title = fields
                yield pid, title, text
    else:
        raise ValueError(f"unknown format {format!r}")


def clean_passage(title: str, text: str, rules: PassageRules) -> Optional[str]:
    """One passage's index text, or None when nothing is left of it
    (build_fm_index.py:74-93)."""
    body = _fix_text(_WHITESPACE.sub(" ", text))
    for marker in _WIKI_MARKERS:
        body = body.replace(marker, "")
    body = body.strip()
    if not body:
        return None
    title = title.strip()
    if rules.word_tokenize is not None:
        title = " ".join(rules.word_tokenize(title))
        body = " ".join(rules.word_tokenize(body))
    if rules.include_title:
        # the reference tests the title after appending the delimiter, so an
        # empty title still contributes " {delim} "
        body = f"{title} {rules.delim} {body}"
    return body.lower() if rules.lowercase else body


def preprocess_file(input_path: str, labels: List[str], format: str = "kilt", lowercase: bool = False,
                    tokenize: bool = False, include_title: bool = False, delim: str = "@@",
                    word_tokenize: Optional[Callable[[str], List[str]]] = None) -> Iterator[str]:
    """build_fm_index.py:52-97: the cleaned passage texts, in file order;
    ``labels`` receives each kept passage's id."""
    if tokenize and word_tokenize is None:
        raise RuntimeError("--tokenize needs a word tokenizer (spacy's English, build_fm_index.py:148-154)")
    rules = PassageRules(include_title, delim, lowercase, word_tokenize if tokenize else None)
    with open(input_path, "r", 2 ** 16) as f:
        for pid, title, text in read_records(f, format):
            cleaned = clean_passage(title, text, rules)
            if cleaned is not None:
                labels.append(pid.strip())
                yield cleaned


# -- tokenization (build_fm_index.py:25-50): one tokenizer per pool worker ----
_worker_tokenizer = None


def init_worker(model_name: Optional[str]) -> None:
    """Pool initializer: load the worker's tokenizer (local files only)."""
    global _worker_tokenizer
    if model_name is None:
        raise RuntimeError("the reference's default tokenizer is fairseq BART from torch.hub, which needs the "
                           "network; pass --hf_model <local tokenizer path or cached name>")
    from transformers import AutoTokenizer

    _worker_tokenizer = AutoTokenizer.from_pretrained(model_name, use_fast=False)


def encode_passage(tokenizer, text: str, bart: bool = False) -> List[int]:
    """Token ids of one passage: ``"Paraphrase: "`` + text (a leading space
    first for BART vocabularies), no special tokens, then eos
    (build_fm_index.py:40-48)."""
    prompt = "Paraphrase: " + (" " if bart else "") + text.strip()
    target = getattr(tokenizer, "as_target_tokenizer", None)
    with (target() if target is not None else contextlib.nullcontext()):
        ids = tokenizer(prompt, add_special_tokens=False)["input_ids"]
    return [*ids, tokenizer.eos_token_id]


def process(line: str, model_name: Optional[str]) -> List[int]:
    """The pool's map function (build_fm_index.py:37)."""
    return encode_passage(_worker_tokenizer, line, bart=model_name is not None and "bart" in model_name)


class CorpusBuffer:
    """T' (index.py:47-53) built incrementally: each appended doc is stored
    reversed with ids + SHIFT in one growing uint32 buffer; ``beginnings`` and
    the set of occurring ids are kept alongside."""

    def __init__(self, capacity: int = 1 << 20):
        self.buf = np.empty(max(16, capacity), dtype=np.uint32)
        self.n = 0
        self.beginnings = [0]
        self.seen = np.zeros(1 << 17, dtype=bool)

    def append(self, seq: Sequence[int]) -> None:
        a = np.asarray(seq, dtype=np.int64)
        if a.size and (int(a.min()) + SHIFT < 1 or int(a.max()) + SHIFT >= (1 << 31)):
            raise OverflowError("token id outside [-9, 2^31 - 11) cannot be encoded")
        need = self.n + a.size + 1
        if need > self.buf.size:
            grown = np.empty(max(need, 2 * self.buf.size), dtype=np.uint32)
            grown[: self.n] = self.buf[: self.n]
            self.buf = grown
        self.buf[self.n: self.n + a.size] = (a[::-1] + SHIFT).astype(np.uint32)
        self.n += a.size
        self.beginnings.append(self.n)
        if a.size:
            top = int(a.max()) + 1
            if top > self.seen.size:
                grown = np.zeros(max(top, 2 * self.seen.size), dtype=bool)
                grown[: self.seen.size] = self.seen
                self.seen = grown
            self.seen[a[a >= 0]] = True
            neg = a[a < 0]
            if neg.size:
                self.neg = set(getattr(self, "neg", set())) | set(neg.tolist())

    @property
    def occurring(self) -> set:
        occ = set(np.flatnonzero(self.seen).tolist())
        return occ | set(getattr(self, "neg", set()))

    def text(self) -> np.ndarray:
        """T' with the sentinel 0 appended (sdsl construct_im adds it)."""
        out = np.empty(self.n + 1, dtype=np.uint32)
        out[: self.n] = self.buf[: self.n]
        out[self.n] = 0
        return out


def index_from_sequences(sequences: Iterable[Sequence[int]], device: Optional[int] = None) -> FMIndex:
    """FMIndex.initialize(sequences) (index.py:39-67) through the streaming
    encoder and the device build: the same index, no host suffix sorting."""
    import torch

    corpus = CorpusBuffer()
    for seq in sequences:
        corpus.append(seq)
    index = FMIndex(device=device)
    dev = torch.device("cuda", index.device)
    text = torch.from_numpy(corpus.text().view(np.int32)).to(dev)
    index.initialize_from_text_device(text, keep_sa_text=True)   # SA kept only to sample it (locate / get_doc)
    del text
    index.beginnings = corpus.beginnings
    index.occurring = sorted(corpus.occurring)
    index.occurring_distinct, index.occurring_counts = index.get_distinct_count(0, len(index))
    return index


def build_index(input_path: str, hf_model: Optional[str] = None, jobs: int = 1, format: str = "kilt",
                lowercase: bool = False, tokenize: bool = False, include_title: bool = False, delim: str = "@@",
                encode: Optional[Callable[[str], List[int]]] = None, device: Optional[int] = None) -> FMIndex:
    """build_fm_index.py:100-114.  ``encode`` (text -> token ids) replaces the
    worker pool's HF tokenizer when given (tests, custom tokenizers)."""
    labels: List[str] = []
    word_tokenize = None
    if tokenize:
        from spacy.lang.en import English   # build_fm_index.py:148-154

        nlp = English()

        def word_tokenize(text):
            return [t.text.strip() for t in nlp.tokenizer(text)]
    lines = preprocess_file(input_path, labels, format, lowercase=lowercase, tokenize=tokenize,
                            include_title=include_title, delim=delim, word_tokenize=word_tokenize)
    if encode is not None:
        index = index_from_sequences((encode(t) for t in lines), device=device)
    else:
        with multiprocessing.Pool(jobs, initializer=init_worker, initargs=(hf_model,)) as pool:
            index = index_from_sequences(pool.imap(partial(process, model_name=hf_model), lines, chunksize=256),
                                         device=device)
    index.labels = labels
    return index


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Build an FM-index (build_fm_index.py) on the GPU")
    p.add_argument("input")
    p.add_argument("output")
    p.add_argument("--jobs", type=int, default=1)
    p.add_argument("--include_title", action="store_true")
    p.add_argument("--delim", default="@@")
    p.add_argument("--format", choices=["kilt", "dpr"], default="kilt")
    p.add_argument("--hf_model", default=None, type=str)
    p.add_argument("--lowercase", action="store_true")
    p.add_argument("--tokenize", action="store_true")
    p.add_argument("--device", type=int, default=None)
    return p.parse_args(argv)


def main(argv=None) -> None:
    args = parse_args(argv)
    print(args)
    index = build_index(args.input, hf_model=args.hf_model, jobs=args.jobs, format=args.format,
                        lowercase=args.lowercase, tokenize=args.tokenize, include_title=args.include_title,
                        delim=args.delim, device=args.device)
    index.save(args.output)


if __name__ == "__main__":
    main()
