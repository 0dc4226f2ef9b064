"""Probe (graph-timed): LF latency vs index size; wide-row mask cost vs B0 / slice width."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
from bench import build_index  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
V, B, R = 128256, 256, 20


def gtime(fn, reps=R):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for n_tok, b0 in [(2e7, 13), (3e8, 13), (3e8, 11)]:
    os.environ["FMIDX_BM_LOG2"] = str(b0)
    fm, text, bwt, _ = build_index(int(n_tok), V, 1, dev)
    n = bwt.numel()
    del text
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    out_lo = torch.empty(B, dtype=torch.int64, device=dev)
    out_hi = torch.empty(B, dtype=torch.int64, device=dev)
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    for w in [1, 1000, 1_000_000]:
        lo = torch.randint(0, n - w - 1, (B,), generator=gen, device=dev)
        hi = lo + w
        tok = bwt[lo].to(torch.int64) - 10
        us = gtime(lambda: fm.lf_step_batch(tok, lo, hi, 10, lo_out=out_lo, hi_out=out_hi))
        print(f"n={n:.1e} B0=2^{b0} LF width {w:>8}: {us:6.1f} us")
    for w in [1, 4, 16384, 1_000_000, 20_000_000]:
        lo = torch.randint(0, n - w - 1, (B,), generator=gen, device=dev)
        hi = lo + w
        for sw in [4096, 16032, 32768]:
            os.environ["FMIDX_MASK_SW"] = str(sw)
            us = gtime(lambda: fm.allowed_mask(lo, hi, V, 10, out=mask))
            print(f"n={n:.1e} B0=2^{b0} mask width {w:>9} SW {sw:>6}: {us:6.1f} us  {B * V / us / 1e3:6.0f} GB/s writes")
        os.environ.pop("FMIDX_MASK_SW")
    del fm, bwt
    torch.cuda.empty_cache()
