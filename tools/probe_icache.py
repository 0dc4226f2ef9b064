"""How much of the cold step is instruction fetch?  A 20-step decode graph on a
large index is replayed after a 1 GiB cache eviction (cold, as bench.py
times it), and after the same eviction followed by one decode step on a tiny
index -- the same kernel, so its code is back in L2 / the Infinity Cache while
the large index, row state and masks are still cold.  The difference is what
fetching the kernel's code from HBM costs the first step of the graph (the
later steps hit L2 either way).  Usage: python tools/probe_icache.py [tokens]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

from fmidx.fm_index import FMIndex  # noqa: E402
from fmidx.synth import decode_trace, markov_corpus_gpu  # noqa: E402

dev = torch.device("cuda", 0)
V, B, W, SHIFT = 128256, 256, 5, 10
K = int(os.environ.get("STEPS", "20"))
flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)


def build(tok, seed):
    text, beg = markov_corpus_gpu(int(tok), V, seed, dev)
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text)
    bwt = fm.device_bwt()
    tokens, init, _, _, _ = decode_trace(fm, text, bwt, B, V, W + K, 1, dev)
    del text
    return fm, tokens, init


big, tokens, init = build(float(sys.argv[1]) if len(sys.argv) > 1 else 4.5e9, 20250905)
small, stok, sinit = build(1e5, 7)
mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
smask = torch.empty((B, V), dtype=torch.uint8, device=dev)
bufs = [(init[0].clone(), init[1].clone()), (torch.empty_like(init[0]), torch.empty_like(init[1]))]
sb = [(sinit[0].clone(), sinit[1].clone()), (torch.empty_like(sinit[0]), torch.empty_like(sinit[1]))]
for i in range(2):
    big.decode_step(tokens[i], bufs[0][0], bufs[0][1], mask, V, SHIFT, reset_below=0,
                    lo_out=bufs[1][0], hi_out=bufs[1][1])
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for i in range(K):
        src, dst = bufs[i % 2], bufs[(i + 1) % 2]
        big.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0, lo_out=dst[0], hi_out=dst[1])


def small_step():
    small.decode_step(stok[W], sb[0][0], sb[0][1], smask, V, SHIFT, reset_below=0, lo_out=sb[1][0], hi_out=sb[1][1])


def timed(pre, reps=5):
    out = []
    for _ in range(reps):
        pre()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / K)
    out.sort()
    return out[len(out) // 2]


cold = timed(lambda: flush.add_(1))
code_warm = timed(lambda: (flush.add_(1), small_step()))
warm = timed(lambda: None)
print(f"K={K}: cold {cold:.2f} us/step, cold data + code in L2 {code_warm:.2f} us/step, warm {warm:.2f} us/step; "
      f"code fetch from HBM ~ {(cold - code_warm) * K:.1f} us per graph (first step)", flush=True)
