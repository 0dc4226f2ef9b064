"""How much of a wide row's mask could be written before its LF step ends?

A decode step's new range for token t lies inside t's C-block [C[t], C[t+1]),
so its allowed set is a subset of t's follow set (the C-block's allowed set):
every 16-token chunk that is all-zero in the follow set is all-zero in the
row's mask and could be zero-filled as soon as t is known (the state's round
trip), leaving only the follow set's non-zero chunks for the late emit.  This
measures, over the bench's C3 trace, for the rows whose new range is wide
(>= 4096 rows: the cached rows whose 128-KB emit ends the step), the fraction
of 16-token chunks that are zero in t's follow set, and (the ceiling of any
subset rule) in the row's own mask.
usage: python tools/follow_density.py [--tokens 4.5e9]
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
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V, B, W, K, SHIFT = 128256, 256, 5, 20, bench.SHIFT
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    tokens, init, lo_hist, hi_hist, _ = decode_trace(fm, text, bwt, B, V, W + K, 20250905, dev)
    del text
    torch.cuda.empty_cache()
    n = fm.size()
    zf, zr, rows, viol = [], [], 0, 0
    for s in range(W, W + K):
        lo, hi = lo_hist[s], hi_hist[s]
        wide = ((torch.clamp(hi, max=n) - lo) >= 4096) & ~((lo == 0) & (hi >= n))   # (the full range: a restart)
        idx = torch.nonzero(wide).flatten()
        if idx.numel() == 0:
            continue
        t = tokens[s][idx]
        # t's C-block: the range of the one-token pattern [t]
        toks = t.to(torch.int64).contiguous()
        offs = torch.arange(idx.numel() + 1, dtype=torch.int64, device=dev)
        clo = torch.zeros(idx.numel(), dtype=torch.int64, device=dev)
        chi = torch.zeros_like(clo)
        fm.backward_search_batch(toks, offs, SHIFT, clo, chi)
        follow = fm.allowed_mask(clo, chi, V, SHIFT)            # uint8 [rows, V]
        own = fm.allowed_mask(lo[idx].contiguous(), hi[idx].contiguous(), V, SHIFT)
        nch = V // 16
        fz = (follow[:, :nch * 16].view(-1, nch, 16).amax(2) == 0).float().mean(1)
        oz = (own[:, :nch * 16].view(-1, nch, 16).amax(2) == 0).float().mean(1)
        viol += int((((own > 0) & (follow == 0)).any(1)).sum())   # rows not from t's C-block (expected 0)
        zf.append(fz.cpu().numpy())
        zr.append(oz.cpu().numpy())
        rows += idx.numel()
    zf = np.concatenate(zf)
    zr = np.concatenate(zr)
    res = {"wide_rows": int(rows), "wide_rows_per_step": rows / K, "rows_outside_follow_set": viol,
           "follow_zero_chunk_frac": {"mean": float(zf.mean()), "p10": float(np.percentile(zf, 10)),
                                      "median": float(np.median(zf)), "p90": float(np.percentile(zf, 90))},
           "own_zero_chunk_frac": {"mean": float(zr.mean()), "p10": float(np.percentile(zr, 10)),
                                   "median": float(np.median(zr)), "p90": float(np.percentile(zr, 90))}}
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
