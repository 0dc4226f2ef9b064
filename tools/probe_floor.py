"""Floor of the decode step on this GPU: the same launch with every row empty
(no LF work, no gathers -- only the 32.8 MB uint8 mask write, or 4 MB packed),
captured in a HIP graph like bench.py.  usage: python tools/probe_floor.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

from fmidx.fm_index import FMIndex, suffix_sort_device  # noqa: E402
from fmidx.synth import markov_corpus_gpu  # noqa: E402

dev = torch.device("cuda", 0)
B, V, K = int(os.environ.get("FLOOR_B", 256)), 128256, 20
text, _ = markov_corpus_gpu(10_000_000, V, 1, dev)
bwt, _ = suffix_sort_device(text)
fm = FMIndex(device=0)
fm.initialize_from_bwt_device(bwt)
for packed in (False, True):
    mask = (torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev) if packed
            else torch.empty((B, V), dtype=torch.uint8, device=dev))
    tok = torch.full((B,), V + 100, dtype=torch.int64, device=dev)      # unknown id -> empty rows
    lo = [torch.zeros(B, dtype=torch.int64, device=dev) for _ in range(2)]
    hi = [torch.zeros(B, dtype=torch.int64, device=dev) for _ in range(2)]
    for i in range(3):
        fm.decode_step(tok, lo[0], hi[0], mask, V, 10, reset_below=-1, lo_out=lo[1], hi_out=hi[1], packed=packed)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            fm.decode_step(tok, lo[i % 2], hi[i % 2], mask, V, 10, reset_below=-1, lo_out=lo[(i + 1) % 2],
                           hi_out=hi[(i + 1) % 2], packed=packed)
    ts = []
    for r in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / K * 1e3)
    print(f"floor B={B} slices={os.environ.get('FMIDX_TUNING', 'auto')} lib={os.environ.get('FMIDX_LIB', '')[-20:]} "
          f"({'packed' if packed else 'uint8'} mask, all rows empty): {min(ts):.1f} us/step "
          f"(median {sorted(ts)[2]:.1f})", flush=True)
