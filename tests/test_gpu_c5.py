"""C5 on a PAQ-shaped corpus (BASELINE configs[4]: the PAQ index,
B = 512 x beam 4 = 2048 rows), on the GPU.

The PAQ index is built from ~24-token docs, each ``tokenizer("Paraphrase: " +
question) + [eos]`` (/root/reference/build_fm_index.py:46-48): every doc shares
the prefix, so the prefix pattern -- the processors' ``force_decoding_from``
at the nq_open eval shape (lm_eval_vllm_connection.py:34-35) -- has one row per
doc.  Here n = 1.5e9 (fmidx.synth.paq_corpus_gpu, a 3-token stand-in prefix;
no tokenizer offline), and every decode step's ranges and full [2048, 128256]
masks are compared with cpu_ref (oracle/cpu_ref.cpp, the sdsl-faithful
restatement) fed the same tokens, over a trace whose rows start from the
prefix alone, the prefix + question tokens, and random n-grams."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHIFT = 10
V = 128256


@pytest.fixture(scope="module")
def c5():
    import torch

    from fmidx.fm_index import FMIndex
    from fmidx.synth import paq_corpus_gpu
    from oracle.cpu_ref import CpuRef

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    dev = torch.device("cuda:0")
    if torch.cuda.get_device_properties(0).total_memory < (200 << 30):
        pytest.skip("needs a 288 GB MI355X")
    torch.cuda.empty_cache()
    text, beg = paq_corpus_gpu(1_500_000_000, V, 17, dev)
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text)
    bwt = fm.device_bwt()
    ref = CpuRef.from_device_bwt(bwt)
    yield {"fm": fm, "text": text, "bwt": bwt, "beg": beg, "ref": ref, "dev": dev}
    del fm, text, bwt, ref
    torch.cuda.empty_cache()


@pytest.mark.timeout(900)
def test_c5_paq_shape(c5):
    import torch

    from fmidx.synth import PAQ_EOS, PAQ_PREFIX, paq_trace

    fm, text, bwt, beg, ref, dev = c5["fm"], c5["text"], c5["bwt"], c5["beg"], c5["ref"], c5["dev"]
    n = text.numel()
    nd = beg.numel() - 1
    assert 1.4e9 < n < 1.6e9 and 18 < n / nd < 30          # ~24-token docs
    # the prefix pattern has (at least) one occurrence per doc, and eos is always followed by it
    lo, hi = fm.get_range_batch([list(PAQ_PREFIX), [PAQ_EOS], [PAQ_EOS, PAQ_PREFIX[0]]], SHIFT)
    w = (hi.astype(np.int64) - lo.astype(np.int64)).tolist()
    assert w[0] >= nd and w[1] == nd and w[2] == nd - 1       # the last doc's eos ends F
    # the decode trace at B = 2048: ranges and full masks == cpu_ref every step
    B, S = 2048, 4
    tokens, init, lo_h, hi_h, pats0 = paq_trace(fm, text, bwt, beg, B, V, S, 505, dev)
    assert sum(1 for p in pats0 if p[:3] == list(PAQ_PREFIX)) > B // 2
    clo = init[0].cpu().numpy().astype(np.uint64)
    chi = init[1].cpu().numpy().astype(np.uint64)
    lo = init[0].clone()
    hi = init[1].clone()
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    cmask = np.zeros((B, V), dtype=np.uint8)
    tok_np = tokens.cpu().numpy()
    widths = []
    for s in range(S):
        fm.decode_step(tokens[s], lo, hi, mask, V, SHIFT, reset_below=0)
        ref.decode_step(np.ascontiguousarray(tok_np[s]), SHIFT, 0, clo, chi, cmask, 16)
        assert np.array_equal(lo.cpu().numpy().astype(np.uint64), clo), f"step {s}: ranges"
        assert np.array_equal(hi.cpu().numpy().astype(np.uint64), chi), f"step {s}: ranges"
        bad = np.nonzero((mask.cpu().numpy() != cmask).any(1))[0]
        assert bad.size == 0, f"step {s}: masks differ on rows {bad[:8].tolist()}"
        widths.append(chi.astype(np.int64) - clo.astype(np.int64))
    wall = np.concatenate(widths)
    assert (wall > 1_000_000).any() and ((wall > 0) & (wall <= 512)).any() and (wall == 0).any()
