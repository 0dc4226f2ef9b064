"""Generate the committed golden vectors (run in the build container only).

This script runs the REFERENCE's own Python layer -- ``index.py`` and the
``document_constrained_generation_*`` logits processors from
``/root/reference`` -- unchanged, on top of the oracle's restatement of the
SWIG/sdsl module (``oracle/fm_oracle.py:NaiveFMIndex`` injected as
``cpp_modules.fm_index``) and a behaviour-preserving stub of the absent
third-party base class ``logits_processor_zoo.transformers.base.BaseLogitsProcessor``
(its ``__call__`` runs ``_process``; no reference processor overrides
``_reset`` or reads base-class state).

Only token-level data and outputs are written (``tests/golden/*.json|npz``);
nothing from the reference's sources is copied.  The GPU box never runs this
script (``/root/reference`` does not exist there).

    python tests/golden/make_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle.fm_oracle import NaiveFMIndex, load_naive  # noqa: E402

U64 = (1 << 64) - 1


def install_stubs(reference: str):
    cpp = types.ModuleType("cpp_modules")
    cpp.__path__ = []  # package
    fm = types.ModuleType("cpp_modules.fm_index")
    fm.FMIndex = NaiveFMIndex
    fm.load_FMIndex = load_naive
    sys.modules["cpp_modules"] = cpp
    sys.modules["cpp_modules.fm_index"] = fm

    lpz = types.ModuleType("logits_processor_zoo")
    lpz.__path__ = []
    tr = types.ModuleType("logits_processor_zoo.transformers")
    tr.__path__ = []
    base = types.ModuleType("logits_processor_zoo.transformers.base")

    class BaseLogitsProcessor:  # stub of the third-party base class
        def __init__(self):
            pass

        def __call__(self, input_ids, scores):
            return self._process(input_ids, scores)

    base.BaseLogitsProcessor = BaseLogitsProcessor
    tr.base = base
    lpz.transformers = tr
    sys.modules["logits_processor_zoo"] = lpz
    sys.modules["logits_processor_zoo.transformers"] = tr
    sys.modules["logits_processor_zoo.transformers.base"] = base
    sys.path.insert(0, reference)


# ---------------------------------------------------------------------------
# corpora (token-level; no tokenizer is available offline)
# ---------------------------------------------------------------------------
def markov_corpus(seed: int, n_docs: int, vocab: int, max_len: int, eos: int | None = None):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n_docs):
        length = int(rng.integers(1, max_len + 1))
        tok = int(rng.integers(0, vocab))
        doc = []
        for _ in range(length):
            doc.append(tok)
            # sticky low-entropy chain so that n-grams repeat
            if rng.random() < 0.6:
                tok = (tok * 7 + 3) % vocab
            else:
                tok = int(rng.integers(0, vocab))
        if eos is not None:
            doc.append(eos)
        docs.append(doc)
    return docs


def sample_corpus_docs(reference: str):
    """``test_data/sample_corpus.tsv``.

    faithful: parsed as ``build_fm_index.py:52-97`` does (split on a real tab,
    keep 3-field rows) -> the file uses a literal two-character ``\\t`` so 0
    docs survive.  normalized: literal ``\\t`` -> tab, ``"{title} @@ {text}"``
    (``--include_title``), ``"Paraphrase: "`` prefix and eos (``:46-48``), with a
    deterministic whitespace-word vocabulary standing in for the Llama-3.2-1B
    tokenizer (ids = 100 + rank of the word in sorted order, eos = 2).
    """
    path = os.path.join(reference, "test_data", "sample_corpus.tsv")
    raw = open(path, encoding="utf-8").read()
    faithful = []
    for line in raw.splitlines():
        parts = line.strip().split("\t", 2)
        if len(parts) == 3:
            faithful.append(parts)
    texts = []
    for line in raw.replace("\\t", "\t").splitlines():
        parts = line.strip().split("\t", 2)
        if len(parts) != 3:
            continue
        _, title, text = parts
        text = " ".join(text.split())
        texts.append("Paraphrase: " + f"{title.strip()} @@ {text}")
    words = sorted({w for t in texts for w in t.split()})
    vocab = {w: 100 + i for i, w in enumerate(words)}
    docs = [[vocab[w] for w in t.split()] + [2] for t in texts]
    return len(faithful), docs


# ---------------------------------------------------------------------------
def index_case(ref_index, name, docs, rng, in_memory):
    idx = ref_index.FMIndex()
    idx.initialize(docs, in_memory=in_memory)
    n = idx.size()
    F = []
    for d in reversed(docs):  # forward text that patterns match
        F.extend(d)
    vocab_hi = max([max(d) for d in docs if d] + [1]) + 3

    patterns = [[]]
    for _ in range(60):
        if F:
            s = int(rng.integers(0, len(F)))
            ln = int(rng.integers(1, 9))
            patterns.append(F[s: s + ln])
    for _ in range(20):
        ln = int(rng.integers(1, 5))
        patterns.append([int(x) for x in rng.integers(0, vocab_hi, size=ln)])
    patterns.append([vocab_hi + 100])               # unknown token
    patterns.append([-10])                          # sentinel symbol 0
    if F:
        patterns.append(F[: min(len(F), 40)])       # long true pattern
        patterns.append(F[-5:])
    ranges_out = []
    for p in patterns:
        lo, hi = idx.get_range(p)
        ranges_out.append([p, int(lo), int(hi), int(idx.get_count(p))])

    ranges = [(0, n), (0, len(idx)), (0, 0), (n, n), (3, 2), (0, n + 7), (n - 1, n)]
    for _ in range(40):
        a = int(rng.integers(0, n + 1))
        b = int(rng.integers(a, n + 1))
        ranges.append((a, b))
    for a in range(0, n, max(1, n // 10)):
        ranges.append((a, a + 1))
        ranges.append((a, a + 2))
    for _, lo, hi, _ in ranges_out[:30]:
        ranges.append((lo, hi))
    dc = []
    for a, b in ranges:
        d, c = idx.get_distinct_count(a, b)
        raw = list(idx.distinct_count(a, b))
        dc.append([a, b, d, c, raw, list(idx.get_distinct(a, b))])
    multi_lo = [r[0] for r in ranges[:25]]
    multi_hi = [r[1] for r in ranges[:25]]
    multi = idx.get_distinct_count_multi(multi_lo, multi_hi)

    steps = []
    syms = sorted(set(int(x) for x in idx.bwt.tolist())) + [0, 1, vocab_hi + 50]
    for _ in range(80):
        s = int(rng.choice(syms))
        lo = int(rng.integers(0, n + 1))
        hi = int(rng.integers(0, n + 3))
        steps.append([s, lo, hi, list(idx.backward_search_step(s, lo, hi))])
    for s in syms[:10]:
        steps.append([s, 0, n - 1, list(idx.backward_search_step(s, 0, n - 1))])
        steps.append([s, 0, n + 10, list(idx.backward_search_step(s, 0, n + 10))])

    multi_bs = []
    for p in patterns[1:40]:
        if p and idx.get_count(p) > 0:
            q = [t + ref_index.SHIFT for t in p]
            multi_bs.append([q, list(idx.backward_search_multi(q))])

    locs = [[r, int(idx.locate(r))] for r in range(0, n + 2)]
    extracts = []
    for _ in range(20):
        a = int(rng.integers(0, n + 1))
        b = int(rng.integers(0, n + 3))
        if b > a and min(b, n) <= a:
            continue  # unbounded loop in the reference (fm_index.cpp:184)
        extracts.append([a, b, list(idx.extract_text(a, b))])
    get_docs = [[d, idx.get_doc(d)] for d in range(idx.n_docs)]
    doc_idx = [[r, idx.get_doc_index_from_row(r)] for r in range(0, n)] if n > 1 else []

    return {
        "name": name,
        "in_memory": in_memory,
        "docs": docs,
        "n": n,
        "len": len(idx),
        "n_docs": idx.n_docs,
        "beginnings": idx.beginnings,
        "occurring": sorted(idx.occurring),
        "occurring_distinct": idx.occurring_distinct,
        "occurring_counts": idx.occurring_counts,
        "bwt": [int(x) for x in idx.bwt.tolist()],
        "sa": [int(x) for x in idx.sa.tolist()],
        "get_range": ranges_out,
        "distinct_count": dc,
        "multi": {"lows": multi_lo, "highs": multi_hi,
                  "out": [[list(a), list(b)] for a, b in multi]},
        "backward_search_step": steps,
        "backward_search_multi": multi_bs,
        "locate": locs,
        "extract_text": extracts,
        "get_doc": get_docs,
        "doc_index_from_row": doc_idx,
    }


# ---------------------------------------------------------------------------
QWEN_END = [151645, 198, 151644, 77091, 198]
LLAMA_END = [78191, 128007, 271]
THINK_DONE = [151668, 271]
SYSTEM = [151667, 271, 151668, 271]


def processor_cases(ref_index, reference):
    import torch
    import document_constrained_generation_causal_qwen as qwen
    import document_constrained_generation_causal as causal
    import document_constrained_generation_seq as seq
    import document_constrained_generation_vllm as vllm

    V = 300
    eos, pad = 2, 0
    rng = np.random.default_rng(7)
    docs = markov_corpus(11, 12, 40, 30, eos=eos)
    docs.append([5, 6, 7, 8, 9, 10, 11, 12, 13, 14])
    idx = ref_index.FMIndex()
    idx.initialize(docs, in_memory=True)
    F = []
    for d in reversed(docs):
        F.extend(d)

    arrays = {}
    meta = []

    def true_ngram(ln):
        s = int(rng.integers(0, max(1, len(F) - ln)))
        return F[s: s + ln]

    def gen_rows(kind, B, L):
        rows = []
        for b in range(B):
            r = rng.random()
            if kind == "qwen":
                body_len = L + 3
                if r < 0.15:
                    body = [int(x) for x in rng.integers(0, 40, size=body_len)]   # still thinking
                elif r < 0.3:
                    body = SYSTEM + true_ngram(max(0, body_len - 4))
                else:
                    k = int(rng.integers(0, body_len - 2))
                    body = [int(x) for x in rng.integers(0, 40, size=k)] + THINK_DONE
                    tail = body_len - len(body)
                    t = true_ngram(tail) if rng.random() < 0.7 else [int(x) for x in rng.integers(0, 60, size=tail)]
                    if rng.random() < 0.15 and tail > 0:
                        t = t[:-1] + [rng.choice([eos, pad])]
                    body = body + t
                body = (body + [pad] * body_len)[:body_len]
                rows.append([1, 3, 4] + QWEN_END + body)
            elif kind == "llama":
                if r < 0.2:
                    body = [int(x) for x in rng.integers(0, 60, size=L)]
                else:
                    body = true_ngram(L)
                body = (body + [pad] * L)[:L]
                if rng.random() < 0.15:
                    body[-1] = int(rng.choice([eos, pad]))
                rows.append([9] + LLAMA_END + body)
            else:  # whole generated sequence (vllm / seq)
                body = true_ngram(L) if r < 0.75 else [int(x) for x in rng.integers(0, 60, size=L)]
                body = (body + [pad] * L)[:L]
                if rng.random() < 0.15:
                    body[-1] = int(rng.choice([eos, pad]))
                rows.append(body)
        return rows

    cid = 0
    # --- causal_qwen (primary) ---
    for lrf in (1.0, 2.0):
        for allow_eos in (True, False):
            for fdf in (None, [3]):
                for stop in (0, 2):
                    for L in (1, 3, 6):
                        proc = qwen.IndexBasedLogitsProcessor(
                            index=idx, num_beams=2, min_new_tokens=3, pad_token_id=pad,
                            eos_token_id=eos, force_decoding_from=fdf, stop_at_count=stop,
                            always_allow_eos=allow_eos, length_reward_factor=lrf)
                        rows = gen_rows("qwen", 4, L)
                        ids = torch.tensor(rows, dtype=torch.long)
                        scores = torch.from_numpy(rng.standard_normal((4, V)).astype(np.float32))
                        out = proc(ids, scores.clone())
                        key = f"c{cid}"
                        arrays[key + "_ids"] = ids.numpy()
                        arrays[key + "_scores"] = scores.numpy()
                        arrays[key + "_out"] = out.numpy()
                        meta.append({"id": key, "variant": "causal_qwen", "num_beams": 2,
                                     "min_new_tokens": 3, "pad": pad, "eos": eos,
                                     "force_decoding_from": fdf, "stop_at_count": stop,
                                     "always_allow_eos": allow_eos, "lrf": lrf})
                        cid += 1
    # bf16 scores
    proc = qwen.IndexBasedLogitsProcessor(index=idx, num_beams=1, min_new_tokens=2, pad_token_id=pad,
                                          eos_token_id=eos, always_allow_eos=True, length_reward_factor=2.0)
    rows = gen_rows("qwen", 3, 5)
    ids = torch.tensor(rows, dtype=torch.long)
    scores = torch.from_numpy(rng.standard_normal((3, V)).astype(np.float32)).to(torch.bfloat16)
    out = proc(ids, scores.clone())
    key = f"c{cid}"
    arrays[key + "_ids"] = ids.numpy()
    arrays[key + "_scores"] = scores.float().numpy()
    arrays[key + "_out"] = out.float().numpy()
    meta.append({"id": key, "variant": "causal_qwen", "num_beams": 1, "min_new_tokens": 2, "pad": pad,
                 "eos": eos, "force_decoding_from": None, "stop_at_count": 0,
                 "always_allow_eos": True, "lrf": 2.0, "dtype": "bfloat16"})
    cid += 1

    # --- causal (llama marker) ---
    for lrf in (1.0, 2.0):
        for allow_eos in (True, False):
            for L in (2, 5):
                proc = causal.IndexBasedLogitsProcessor(
                    index=idx, num_beams=2, model_name="llama-3", pad_token_id=pad, eos_token_id=eos,
                    always_allow_eos=allow_eos, length_reward_factor=lrf)
                rows = gen_rows("llama", 4, L)
                ids = torch.tensor(rows, dtype=torch.long)
                scores = torch.from_numpy(rng.standard_normal((4, V)).astype(np.float32))
                out = proc(ids, scores.clone())
                key = f"c{cid}"
                arrays[key + "_ids"] = ids.numpy()
                arrays[key + "_scores"] = scores.numpy()
                arrays[key + "_out"] = out.numpy()
                meta.append({"id": key, "variant": "causal", "model_name": "llama-3", "num_beams": 2,
                             "pad": pad, "eos": eos, "always_allow_eos": allow_eos, "lrf": lrf,
                             "force_decoding_from": None, "stop_at_count": 0})
                cid += 1

    # --- vllm (hard mask, one sequence per call) ---
    for allow_eos in (True, False):
        for L in (1, 2, 4, 7):
            for rep in range(3):
                proc = vllm.IndexBasedLogitsProcessor(index=idx, num_beams=1, pad_token_id=pad, eos_token_id=eos,
                                                      always_allow_eos=allow_eos)
                row = gen_rows("vllm", 1, L)[0]
                scores = torch.from_numpy(rng.standard_normal((V,)).astype(np.float32))
                out = proc(tuple(row), scores.clone())
                key = f"c{cid}"
                arrays[key + "_ids"] = np.asarray([row], dtype=np.int64)
                arrays[key + "_scores"] = scores.numpy()[None]
                arrays[key + "_out"] = out.numpy()
                meta.append({"id": key, "variant": "vllm", "num_beams": 1, "pad": pad, "eos": eos,
                             "always_allow_eos": allow_eos, "force_decoding_from": None, "stop_at_count": 0})
                cid += 1
    # empty generation for vllm
    proc = vllm.IndexBasedLogitsProcessor(index=idx, num_beams=1, pad_token_id=pad, eos_token_id=eos)
    scores = torch.from_numpy(rng.standard_normal((V,)).astype(np.float32))
    out = proc(tuple(), scores.clone())
    key = f"c{cid}"
    arrays[key + "_ids"] = np.zeros((1, 0), dtype=np.int64)
    arrays[key + "_scores"] = scores.numpy()[None]
    arrays[key + "_out"] = out.numpy()
    meta.append({"id": key, "variant": "vllm", "num_beams": 1, "pad": pad, "eos": eos,
                 "always_allow_eos": False, "force_decoding_from": None, "stop_at_count": 0})
    cid += 1

    # --- seq2seq (hard mask, decoder start token skipped) ---
    for allow_eos in (True, False):
        for L in (1, 2, 5):
            proc = seq.IndexBasedLogitsProcessor(index=idx, num_beams=2, pad_token_id=pad, eos_token_id=eos,
                                                 always_allow_eos=allow_eos)
            rows = [[pad] + r for r in gen_rows("seq", 4, L)] if L > 1 else [[pad]] * 4
            ids = torch.tensor(rows, dtype=torch.long)
            scores = torch.from_numpy(rng.standard_normal((4, V)).astype(np.float32))
            out = proc(ids, scores.clone())
            key = f"c{cid}"
            arrays[key + "_ids"] = ids.numpy()
            arrays[key + "_scores"] = scores.numpy()
            arrays[key + "_out"] = out.numpy()
            meta.append({"id": key, "variant": "seq", "num_beams": 2, "pad": pad, "eos": eos,
                         "always_allow_eos": allow_eos, "force_decoding_from": None, "stop_at_count": 0})
            cid += 1

    return {"docs": docs, "vocab": V, "cases": meta}, arrays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default=os.environ.get("FM_REFERENCE", "/root/reference"))
    args = ap.parse_args()
    install_stubs(args.reference)
    import index as ref_index  # the reference's own index.py

    rng = np.random.default_rng(20250905)
    cases = []
    cases.append(index_case(ref_index, "toy_2docs", [[1, 2, 3], [2, 3, 4]], rng, True))
    cases.append(index_case(ref_index, "toy_file_path", [[1, 2, 3], [2, 3, 4]], rng, False))
    cases.append(index_case(ref_index, "single_token", [[7]], rng, True))
    cases.append(index_case(ref_index, "repeats", [[1] * 9, [1, 1, 2], [2, 1]], rng, True))
    cases.append(index_case(ref_index, "with_empty_doc", [[3, 4], [], [4, 3, 4]], rng, True))
    cases.append(index_case(ref_index, "markov_small", markov_corpus(1, 15, 24, 25, eos=2), rng, True))
    cases.append(index_case(ref_index, "markov_mid", markov_corpus(2, 60, 200, 80, eos=2), rng, False))
    cases.append(index_case(ref_index, "sparse_128k",
                            [[int(x) for x in np.random.default_rng(3).integers(0, 128256, size=50)]
                             for _ in range(6)] + [[128255, 0, 1, 128255, 0]], rng, True))
    n_faithful, norm_docs = sample_corpus_docs(args.reference)
    c1 = index_case(ref_index, "sample_corpus_normalized", norm_docs, rng, False)
    c1["faithful_docs"] = n_faithful
    cases.append(c1)
    # the faithful parse yields 0 docs -> an index over the sentinel only
    empty = ref_index.FMIndex()
    try:
        empty.initialize([], in_memory=True)
        cases.append({"name": "sample_corpus_faithful_empty", "n": empty.size(), "len": len(empty),
                      "occurring_distinct": empty.occurring_distinct,
                      "get_range": [[p, *empty.get_range(p), empty.get_count(p)] for p in ([], [5], [0, 1])]})
    except Exception as e:  # pragma: no cover
        print("empty index:", e)

    with open(os.path.join(HERE, "index_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f, separators=(",", ":"))

    pmeta, arrays = processor_cases(ref_index, args.reference)
    with open(os.path.join(HERE, "processor_cases.json"), "w") as f:
        json.dump(pmeta, f, separators=(",", ":"))
    np.savez_compressed(os.path.join(HERE, "processor_cases.npz"), **arrays)
    print("wrote", len(cases), "index cases,", len(pmeta["cases"]), "processor cases")


if __name__ == "__main__":
    main()
