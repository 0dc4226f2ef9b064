"""End to end through Hugging Face ``generate``: a causal LM (random weights)
decodes under the engine's hard-mask processor (the reference's
``document_constrained_generation_seq.py`` semantics: pattern = generated
tokens after the first, -inf outside the allowed set) plugged in through
``LogitsProcessorList`` exactly as the reference's drivers do
(``index_for_transformers_seq.py``).  Every generated continuation must then
be an n-gram of the indexed text F (docs concatenated in reverse order,
SURVEY §8 notation) -- the guarantee constrained decoding exists for."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BOS, EOS, PAD, V = 61, 62, 63, 64


def _docs(seed, n_docs, vocab, max_len):
    rng = np.random.default_rng(seed)
    docs = []
    for _ in range(n_docs):
        ln = int(rng.integers(2, max_len + 1))
        tok = int(rng.integers(0, vocab))
        d = []
        for _ in range(ln):
            d.append(tok)
            tok = (tok * 7 + 3) % vocab if rng.random() < 0.6 else int(rng.integers(0, vocab))
        docs.append(d)
    return docs


def _is_ngram(seq, F):
    n = len(seq)
    if n == 0:
        return True
    a = np.lib.stride_tricks.sliding_window_view(np.asarray(F), n)
    return bool((a == np.asarray(seq)).all(axis=1).any())


@pytest.mark.parametrize("do_sample", [False, True])
def test_generate_under_hard_mask_yields_corpus_ngrams(do_sample):
    import torch
    from transformers import LlamaConfig, LlamaForCausalLM, LogitsProcessorList

    from fmidx.index import FMIndex
    from fmidx.processors import SeqIndexBasedLogitsProcessor

    assert torch.cuda.is_available()
    torch.manual_seed(0)
    docs = _docs(3, 120, 60, 40)
    F = [t for d in reversed(docs) for t in d]
    index = FMIndex(device=0)
    index.initialize(docs, in_memory=True)
    cfg = LlamaConfig(vocab_size=V, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                      num_attention_heads=4, num_key_value_heads=4, max_position_embeddings=64,
                      bos_token_id=BOS, eos_token_id=EOS, pad_token_id=PAD)
    model = LlamaForCausalLM(cfg).cuda().eval()
    proc = SeqIndexBasedLogitsProcessor(index=index, num_beams=1, pad_token_id=PAD, eos_token_id=EOS,
                                        always_allow_eos=True)
    B = 16
    input_ids = torch.full((B, 1), BOS, dtype=torch.long, device="cuda")
    with torch.no_grad():
        out = model.generate(input_ids, attention_mask=torch.ones_like(input_ids), max_new_tokens=12,
                             do_sample=do_sample, top_k=0, logits_processor=LogitsProcessorList([proc]),
                             eos_token_id=EOS, pad_token_id=PAD)
    gen = out[:, 1:].cpu().tolist()
    lengths = []
    for row in gen:
        seq = []
        for t in row:
            if t in (EOS, PAD):
                break
            seq.append(t)
        assert _is_ngram(seq, F), seq
        lengths.append(len(seq))
    assert max(lengths) >= 3       # the constraint is exercised beyond unigrams
