"""Width histogram of the bench's rank pairs (bench.rank_pairs: 2^19 independent
(state, token) LF steps of a C3 decode trace), by the LF kernels' row classes,
and the grouped / sweep launch times on them (cold, median of 3).

usage: python tools/rank_widths.py [--tokens 4.5e9]
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
from fmidx.options import tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--rows", type=int, default=65536)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V = 128256
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    n = fm.size()
    tok, lo, hi, ref = bench.rank_pairs(fm, text, bwt, V, 20250905 + 17, dev, rows=args.rows)
    t = tok.cpu().numpy() + bench.SHIFT
    l = lo.cpu().numpy()
    h = np.minimum(hi.cpu().numpy(), n)
    w = np.where(h > l, h - l, 0)
    live = (t >= 0) & (w > 0)
    full = live & (l == 0) & (h == n)
    edges = [1, 2, 3, 5, 9, 17, 33, 65, 129, 513, 4096, 1 << 40]
    hist = {}
    for a, b in zip(edges[:-1], edges[1:]):
        hist[f"{a}-{b - 1}"] = int(((w >= a) & (w < b) & live & ~full).sum())
    res = {"pairs": int(t.size), "dead": int((~live).sum()), "full": int(full.sum()), "width_hist": hist}
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    ol, oh = torch.empty_like(lo), torch.empty_like(hi)

    def timed(**tun):
        ts = []
        with tuning(**tun):
            for _ in range(4):
                flush.add_(1)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fm.lf_step_batch(tok, lo, hi, bench.SHIFT, lo_out=ol, hi_out=oh, reset_below=0)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
        ok = bool(torch.equal(ol, ref[0]) and torch.equal(oh, ref[1]))
        return {"cold_us": float(np.median(ts[1:])), "exact": ok}

    pc = fm.cache_contains(lo, hi).cpu().numpy().astype(bool)
    classes = {"singleton": live & ~full & (w == 1), "narrow_2_16": live & ~full & (w >= 2) & (w <= 16),
               "e_17_512": live & ~full & (w > 16) & (w <= 512),
               "probe": live & ~full & (w >= (fm.stats()["cache_min"] or 1 << 62)) & pc,
               "descent": live & ~full & (w > 512) & ~pc, "full": full, "dead": ~live}
    res["by_class"] = {}
    for name, sel in classes.items():
        idx = torch.tensor(np.flatnonzero(sel), dtype=torch.int64, device=dev)
        if idx.numel() == 0:
            continue
        t_, l_, h_ = tok[idx].contiguous(), lo[idx].contiguous(), hi[idx].contiguous()
        o1, o2 = torch.empty_like(l_), torch.empty_like(h_)
        ts = []
        for _ in range(4):
            flush.add_(1)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fm.lf_step_batch(t_, l_, h_, bench.SHIFT, lo_out=o1, hi_out=o2, reset_below=0)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        ok = bool(torch.equal(o1, ref[0][idx]) and torch.equal(o2, ref[1][idx]))
        res["by_class"][name] = {"rows": int(idx.numel()), "cold_us": float(np.median(ts[1:])), "exact": ok}
    res["grouped"] = timed(lf_work=0)
    res["sweep_tail"] = timed(lf_work=2)
    res["default"] = timed()
    res["lists"] = timed(lf_work=3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
