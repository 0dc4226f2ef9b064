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
from functools import partial
from typing import Callable, Iterable, Iterator, List, Optional, Sequence

import numpy as np

from .index import SHIFT, FMIndex

try:                                    # build_fm_index.py:13
    from ftfy import fix_text as _fix_text
except ImportError:                     # pragma: no cover - not in this image
    def _fix_text(text: str) -> str:
        return text


def preprocess_file(input_path: str, labels: List[str], format: str = "kilt", lowercase: bool = False,
                    tokenize: bool = False, include_title: bool = False, delim: str = "@@",
                    word_tokenize: Optional[Callable[[str], List[str]]] = None) -> Iterator[str]:
    """build_fm_index.py:52-97: the cleaned passage texts, in file order;
    ``labels`` receives each kept passage's id."""
    with open(input_path, "r", 2 ** 16) as f:
        if format == "dpr":
            next(f)
            rows = csv.reader(f, delimiter="\t", quotechar='"')
            pieces = ((pp[0], pp[2], pp[1]) for pp in rows if len(pp) == 3)
        elif format == "kilt":
            lines = (line.strip() for line in f)
            split = (line.split("\t", 2) for line in lines)
            pieces = ((pp[0], pp[1], pp[2]) for pp in split if len(pp) == 3)
        else:
            raise ValueError(f"unknown format {format!r}")
        for idx, title, text in pieces:
            idx = idx.strip()
            title = title.strip()
            text = re.sub(r"\s+", " ", text)
            text = _fix_text(text)
            text = text.replace("BULLET::::", "")
            text = text.replace("SECTION::::", "")
            text = text.strip()
            if not text:
                continue
            if tokenize:
                if word_tokenize is None:
                    raise RuntimeError("--tokenize needs a word tokenizer (spacy's English, build_fm_index.py:148-154)")
                title = " ".join(word_tokenize(title))
                text = " ".join(word_tokenize(text))
            title = f"{title} {delim}"
            if include_title and title:
                text = f"{title} {text}"
            if lowercase:
                text = text.lower()
            labels.append(idx)
            yield text


# -- tokenization (build_fm_index.py:25-50), one tokenizer per worker ---------
_tokenizer = None


def init_worker(model_name: Optional[str]) -> None:
    global _tokenizer
    if model_name is None:
        raise RuntimeError("the reference's default tokenizer is fairseq BART from torch.hub, which needs the "
                           "network; pass --hf_model <local tokenizer path or cached name>")
    from transformers import AutoTokenizer

    _tokenizer = AutoTokenizer.from_pretrained(model_name, use_fast=False)


def process(line: str, model_name: Optional[str]) -> List[int]:
    is_bart = model_name is not None and "bart" in model_name
    line = line.strip()
    if is_bart:
        line = " " + line
    ctx = getattr(_tokenizer, "as_target_tokenizer", None)
    with (ctx() if ctx is not None else contextlib.nullcontext()):
        line = "Paraphrase: " + line
        return list(_tokenizer(line, add_special_tokens=False)["input_ids"]) + [_tokenizer.eos_token_id]


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
