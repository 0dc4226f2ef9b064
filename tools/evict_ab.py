"""How the cache eviction before a cold timed region shapes the cold figure.

The bench evicts with a 1 GiB read-modify-write (flush.add_(1)): that leaves up
to the 256 MB MALL full of DIRTY lines of an unrelated buffer, which the timed
kernels then have to write back as their own traffic evicts them.  Here the
bench's K = 20 decode graph and the 2^19-pair rank launch are timed cold after
  rmw        -- the bench's eviction (read-modify-write of 1 GiB), then sync;
  read       -- a 1 GiB read-only pass (a sum: the caches end up holding clean
                lines of the flush buffer), then sync;
  rmw+read   -- the read-modify-write, then the read-only pass (the dirty lines
                are written back before the timed region), then sync;
each R times, interleaved, plus warm.
usage: python tools/evict_ab.py [--tokens 4.5e9] [--reps 7]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx.synth import decode_trace  # noqa: E402

SHIFT = bench.SHIFT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V, B, W, K = 128256, 256, 5, 20
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    tokens, init, lo_hist, hi_hist, _ = decode_trace(fm, text, bwt, B, V, W + K, 20250905, dev)
    rtok, rlo, rhi, rref = bench.rank_pairs(fm, text, bwt, V, 20250905 + 17, dev)
    del text
    torch.cuda.empty_cache()
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    lo, hi = init[0].clone(), init[1].clone()
    for s in range(W):
        fm.decode_step(tokens[s], lo, hi, mask, V, SHIFT, reset_below=0)
    st_lo, st_hi = lo.clone(), hi.clone()
    bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            src, dst = bufs[i % 2], bufs[(i + 1) % 2]
            fm.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0,
                           lo_out=dst[0], hi_out=dst[1])
    olo, ohi = torch.empty_like(rlo), torch.empty_like(rhi)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        fm.lf_step_batch(rtok, rlo, rhi, SHIFT, lo_out=olo, hi_out=ohi, reset_below=0)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    acc = torch.zeros((), dtype=torch.int64, device=dev)

    def evict(kind):
        if kind in ("rmw", "rmw+read"):
            flush.add_(1)
        if kind in ("read", "rmw+read"):
            torch.sum(flush, 0, dtype=torch.int64, out=acc)

    def timed(replay, kind, per):
        if kind == "warm":
            lo.copy_(st_lo)
            hi.copy_(st_hi)
            replay()
        else:
            evict(kind)
        lo.copy_(st_lo)     # the decode graph always starts from the trace's state
        hi.copy_(st_hi)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / per

    kinds = ("rmw", "read", "rmw+read", "warm")
    res = {"decode_us_per_step": {k: [] for k in kinds}, "rank_2_19_us": {k: [] for k in kinds}}
    for _ in range(args.reps):
        for k in kinds:
            res["decode_us_per_step"][k].append(timed(g.replay, k, K))
            res["rank_2_19_us"][k].append(timed(gr.replay, k, 1))
    fin = bufs[K % 2]
    res["trace_ok"] = bool(torch.equal(fin[0], lo_hist[W + K - 1]) and torch.equal(fin[1], hi_hist[W + K - 1]))
    res["rank_exact"] = bool(torch.equal(olo, rref[0]) and torch.equal(ohi, rref[1]))
    res["median"] = {f"{w}:{k}": float(np.median(res[w][k])) for w in ("decode_us_per_step", "rank_2_19_us")
                     for k in kinds}
    print(json.dumps(res["median"]), flush=True)
    print(json.dumps({"trace_ok": res["trace_ok"], "rank_exact": res["rank_exact"]}), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
