"""Kernel probe: time k_mask / k_lf on controlled row mixes (HIP events,
back-to-back launches).  Usage: python tools/probe_kernels.py [--tokens 3e8]"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
from bench import build_index  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=float, default=3e8)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--reps", type=int, default=20)
args = ap.parse_args()
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
V, B, R = 128256, args.batch, args.reps
fm, text, bwt, _ = build_index(int(args.tokens), V, 1, dev)
n = bwt.numel()
g = torch.Generator(device=dev)
g.manual_seed(5)


def ranges(width):
    lo = torch.randint(0, n - width - 1, (B,), generator=g, device=dev)
    return lo, lo + width


mixes = {
    "empty": (torch.zeros(B, dtype=torch.int64, device=dev), torch.zeros(B, dtype=torch.int64, device=dev)),
    "w1": ranges(1),
    "w8": ranges(8),
    "w1k": ranges(1000),
    "w16k": ranges(16384),
    "w1M": ranges(1_000_000),
    "full": (torch.zeros(B, dtype=torch.int64, device=dev), torch.full((B,), n, dtype=torch.int64, device=dev)),
}
lo, hi = ranges(4)
lo[::10] = 0
hi[::10] = n
mixes["w4+10%full"] = (lo, hi)
mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
packed = torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev)
print(f"n={n} B={B} V={V} stats={fm.stats()}")


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(R):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / R * 1e3


for name, (lo, hi) in mixes.items():
    us = timeit(lambda: fm.allowed_mask(lo, hi, V, 10, out=mask))
    usp = timeit(lambda: fm.allowed_mask(lo, hi, V, 10, out=packed, packed=True))
    print(f"mask {name:12s} {us:8.1f} us  ({B * V / us / 1e3:7.0f} GB/s of writes)   packed {usp:8.1f} us")

# LF: live rows stepping by a true next symbol
for name, (lo, hi) in [("w1", mixes["w1"]), ("w1k", mixes["w1k"]), ("full", mixes["full"]), ("empty", mixes["empty"])]:
    j = lo.clamp(max=n - 1)
    tok = bwt[j].to(torch.int64) - 10
    lo2, hi2 = lo.clone(), hi.clone()

    def f():
        lo2.copy_(lo)
        hi2.copy_(hi)
        fm.lf_step_batch(tok, lo2, hi2, 10)
    us = timeit(f)
    print(f"lf   {name:12s} {us:8.1f} us")
