"""Cold vs warm cost of one fused decode step, by what the step reads.
K = 20 steps in a HIP graph, timed after a 1 GiB cache eviction (cold) and
back to back (warm), as bench.py does, for: (a) every row empty (no index read:
the row state, the code and the 33 MB of mask stores only), (b) the bench's
trace on a 1e6-token index (index data a few MB), (c) the trace on a 1.5e9 /
4.5e9-token index.  Usage: python tools/probe_cold.py [tokens...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

from fmidx.fm_index import FMIndex  # noqa: E402
from fmidx.synth import decode_trace, markov_corpus_gpu  # noqa: E402

dev = torch.device("cuda", 0)
V, B, K, W, SHIFT = 128256, 256, 20, 5, 10
flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)


def timed(g, cold, reps=3):
    out = []
    for _ in range(reps):
        if cold:
            flush.add_(1)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / K)
    return min(out)


def run(name, fm, tokens, lo0, hi0, packed=False):
    mask = (torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev) if packed
            else torch.empty((B, V), dtype=torch.uint8, device=dev))
    bufs = [(lo0.clone(), hi0.clone()), (torch.empty_like(lo0), torch.empty_like(hi0))]
    for i in range(2):   # warm up the code path once
        fm.decode_step(tokens[i], bufs[0][0], bufs[0][1], mask, V, SHIFT, reset_below=0,
                       lo_out=bufs[1][0], hi_out=bufs[1][1], packed=packed)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            src, dst = bufs[i % 2], bufs[(i + 1) % 2]
            fm.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0,
                           lo_out=dst[0], hi_out=dst[1], packed=packed)
    c, w = timed(g, True), timed(g, False)
    print(f"{name:34s} cold {c:6.2f} us/step  warm {w:6.2f} us/step  (+{c - w:.2f})", flush=True)


for tok in [float(x) for x in (sys.argv[1:] or ["1e6", "1.5e9"])]:
    text, beg = markov_corpus_gpu(int(tok), V, 20250905, dev)
    fm = FMIndex(device=0)
    fm.initialize_from_text_device(text)
    bwt = fm.device_bwt()
    tokens, init, _, _, _ = decode_trace(fm, text, bwt, B, V, W + K, 1, dev)
    del text
    z = torch.zeros(B, dtype=torch.int64, device=dev)
    dead = torch.full_like(tokens, 5)                     # every row empty: tokens never restart
    run(f"n={tok:.0e} all rows empty", fm, dead, z, z)
    run(f"n={tok:.0e} all rows empty packed", fm, dead, z, z, packed=True)
    run(f"n={tok:.0e} trace", fm, tokens, init[0], init[1])
    run(f"n={tok:.0e} trace packed", fm, tokens, init[0], init[1], packed=True)
    del fm, bwt, tokens
    torch.cuda.empty_cache()
