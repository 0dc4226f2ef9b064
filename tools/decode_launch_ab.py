"""How the timed decode steps are launched: one K-step graph replay (the bench)
against K direct launches, cold (after the bench's 1 GiB eviction), same trace.

  graph        -- the K steps captured in one HIP graph, replayed after the eviction
                  has completed (the bench's timed region);
  direct_sync  -- the K steps launched directly (fm_decode_step_batch per step, as
                  the processors launch them) after the eviction has completed: the
                  host's per-launch cost is inside the events when it exceeds a kernel;
  direct_queued-- the same K launches enqueued behind the eviction while it runs.
Interleaved repetitions, median per step; every mode's final state checked.
usage: python tools/decode_launch_ab.py [--tokens 4.5e9] [--reps 5] [--out f.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V, B, W, K, SHIFT = 128256, 256, 5, args.steps, bench.SHIFT
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    tokens, init, lo_hist, hi_hist, _ = decode_trace(fm, text, bwt, B, V, W + K, 20250905, dev)
    del text
    torch.cuda.empty_cache()
    mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    lo, hi = init[0].clone(), init[1].clone()
    for s in range(W):
        fm.decode_step(tokens[s], lo, hi, mask, V, SHIFT, reset_below=0)
    torch.cuda.synchronize()
    st_lo, st_hi = lo.clone(), hi.clone()
    bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]

    def steps():
        for i in range(K):
            src, dst = bufs[i % 2], bufs[(i + 1) % 2]
            fm.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0, lo_out=dst[0], hi_out=dst[1])

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        steps()
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)

    def one(mode):
        lo.copy_(st_lo)
        hi.copy_(st_hi)
        torch.cuda.synchronize()
        flush.add_(1)
        if mode != "direct_queued":
            torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        if mode == "graph":
            g.replay()
        else:
            steps()
        b.record()
        torch.cuda.synchronize()
        fin = bufs[K % 2]
        ok = bool(torch.equal(fin[0], lo_hist[W + K - 1]) and torch.equal(fin[1], hi_hist[W + K - 1]))
        return a.elapsed_time(b) * 1e3 / K, ok

    modes = ("graph", "direct_sync", "direct_queued")
    for m in modes:   # untimed: first launches
        one(m)
    res = {m: [] for m in modes}
    oks = {m: True for m in modes}
    for _ in range(args.reps):
        for m in modes:
            t, ok = one(m)
            res[m].append(t)
            oks[m] = oks[m] and ok
    out = {"K": K, "B": B, "tokens": int(args.tokens),
           "us_per_step": {m: sorted(v) for m, v in res.items()},
           "median_us_per_step": {m: float(np.median(v)) for m, v in res.items()},
           "exact": oks}
    print(json.dumps(out), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
