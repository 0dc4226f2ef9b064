"""Class-list LF launch (lf_work 3) on subsets of the bench's 2^19 rank pairs,
cold, 4 launches each (for a kernel trace: k_lf_class / k_lf_lists durations
by subset).  usage: python tools/lf_lists_probe.py [--lf-work 3]"""
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
    ap.add_argument("--lf-work", type=int, default=3)
    ap.add_argument("--rows", type=int, default=65536, help="trace rows (pairs = 8 x rows)")
    ap.add_argument("--compare", default="", help="also the 'all' set under these lf_work values, e.g. -1,0")
    ap.add_argument("--split", type=int, default=0, help="also the 'all' set as this many parts on as many streams")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    fm, text, bwt, _ = bench.build_index(int(4.5e9), 128256, 20250905, dev)
    n = fm.size()
    tok, lo, hi, ref = bench.rank_pairs(fm, text, bwt, 128256, 20250905 + 17, dev, rows=args.rows)
    w = torch.clamp(hi, max=n) - lo
    live = (tok + bench.SHIFT >= 0) & (w > 0)
    single = (w == 1) & live
    pc = fm.cache_contains(lo, hi).bool()
    full = live & (lo == 0) & (torch.clamp(hi, max=n) == n)
    probe = live & ~full & (w >= 4096) & pc
    e17 = live & ~full & (w > 16) & (w <= 512)
    desc = live & ~full & (w > 512) & ~pc
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    res = {}
    for name, sel in (("all", None), ("single", single), ("nonsingle", ~single), ("probe", probe), ("e17_512", e17),
                      ("descent", desc)):
        if sel is None:
            t_, l_, h_, r0, r1 = tok, lo, hi, ref[0], ref[1]
        else:
            idx = torch.nonzero(sel).flatten()
            t_, l_, h_, r0, r1 = tok[idx], lo[idx], hi[idx], ref[0][idx], ref[1][idx]
        o1, o2 = torch.empty_like(l_), torch.empty_like(h_)
        ts = []
        with tuning(lf_work=args.lf_work):
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
        res[name] = {"rows": int(t_.numel()), "cold_us": float(np.median(ts[1:])),
                     "exact": bool(torch.equal(o1, r0) and torch.equal(o2, r1))}
    for lw in [int(x) for x in args.compare.split(",") if x.strip()]:
        o1, o2 = torch.empty_like(lo), torch.empty_like(hi)
        ts = []
        with tuning(lf_work=lw):
            for _ in range(4):
                flush.add_(1)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fm.lf_step_batch(tok, lo, hi, bench.SHIFT, lo_out=o1, hi_out=o2, reset_below=0)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
        res[f"all_lf_work{lw}"] = {"cold_us": float(np.median(ts[1:])),
                                   "exact": bool(torch.equal(o1, ref[0]) and torch.equal(o2, ref[1]))}
    if args.split > 1:
        K = args.split
        parts = torch.tensor_split(torch.arange(tok.numel(), device=dev), K)
        ins = [(tok[p].contiguous(), lo[p].contiguous(), hi[p].contiguous()) for p in parts]
        outs = [(torch.empty_like(x[1]), torch.empty_like(x[2])) for x in ins]
        streams = [torch.cuda.Stream(dev) for _ in range(K)]
        for lw in (args.lf_work, 0):
            ts = []
            with tuning(lf_work=lw):
                for _ in range(4):
                    flush.add_(1)
                    torch.cuda.synchronize()
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    a.record()
                    cur = torch.cuda.current_stream(dev)
                    for (t_, l_, h_), (o1, o2), st in zip(ins, outs, streams):
                        st.wait_stream(cur)
                        with torch.cuda.stream(st):
                            fm.lf_step_batch(t_, l_, h_, bench.SHIFT, lo_out=o1, hi_out=o2, reset_below=0)
                    for st in streams:
                        cur.wait_stream(st)
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b) * 1e3)
            ok = all(torch.equal(o[0], ref[0][p]) and torch.equal(o[1], ref[1][p]) for o, p in zip(outs, parts))
            res[f"all_split{K}_lf_work{lw}"] = {"cold_us": float(np.median(ts[1:])), "exact": bool(ok)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
