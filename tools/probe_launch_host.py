"""Host cost of ONE decode-step launch (what a processor pays per step when it
launches eagerly): fm.decode_step through the Python wrapper, its pieces
(the current-stream lookup, the ctypes call with precomputed arguments), and
lf_step_batch -- per call, enqueue only (the GPU is left to drain after the
timed loop), on a small index at B = 256 and B = 32.
usage: python tools/probe_launch_host.py [--calls 2000] [--out f.json]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fmidx._lib import lib  # noqa: E402
from fmidx.fm_index import _stream_of  # noqa: E402
from fmidx.index import FMIndex  # noqa: E402


def per_call(fn, calls):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(calls):
        fn()
    dt = (time.perf_counter() - t) / calls * 1e6
    torch.cuda.synchronize()
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    V = 128256
    docs = [rng.integers(0, V, size=int(rng.integers(50, 400))).tolist() for _ in range(3000)]
    fm = FMIndex(device=0)
    fm.initialize(docs, in_memory=True)
    n = fm.size()
    res = {"n": int(n), "calls": args.calls}
    for B in (256, 32):
        tok = torch.randint(0, V, (B,), dtype=torch.int64, device=dev)
        lo = torch.zeros(B, dtype=torch.int64, device=dev)
        hi = torch.full((B,), n, dtype=torch.int64, device=dev)
        lo2, hi2 = torch.empty_like(lo), torch.empty_like(hi)
        mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
        r = {}
        r["decode_step_us"] = per_call(lambda: fm.decode_step(tok, lo, hi, mask, V, 0, lo_out=lo2, hi_out=hi2), args.calls)
        r["lf_step_batch_us"] = per_call(lambda: fm.lf_step_batch(tok, lo, hi, 0, lo_out=lo2, hi_out=hi2), args.calls)
        r["stream_lookup_us"] = per_call(lambda: _stream_of(lo), args.calls)
        fn = lib().fm_decode_step_batch
        a = (fm._h, tok.data_ptr(), 0, -(1 << 63), lo.data_ptr(), hi.data_ptr(), lo2.data_ptr(), hi2.data_ptr(), B,
             mask.data_ptr(), V, V, 0, _stream_of(lo))
        r["ctypes_call_only_us"] = per_call(lambda: fn(*a), args.calls)
        # the C++ entry with every argument prebuilt as a ctypes object
        ca = [fm._h] + [ctypes.c_void_p(x) if i in (1, 4, 5, 6, 7, 9, 13) else x for i, x in enumerate(a) if i > 0]
        r["ctypes_prebuilt_us"] = per_call(lambda: fn(*ca), args.calls)
        res[f"B{B}"] = r
        print(B, json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
