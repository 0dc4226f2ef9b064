"""Tail rows of the in-wave LF sweep (k_lf_sweep<true>) per wave, on the
bench's 2^19 and 2^21 rank pairs: which rows the sweep cannot settle in its
packed E scan or its probe batches, by kind, and how many land in each wave of
64 consecutive rows (the rows a wave then steps one at a time).
  T1  an E scan of 65..512 rows (lf_step_fast by the whole wave)
  T2  a descent: an uncached range > 512 rows, or a cached range whose probe
      missed (an absent symbol ends after the descent's first level)
usage: python tools/tail_hist.py [--tokens 4.5e9]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V = 128256
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    n = fm.size()
    st = fm.stats()
    cache_min = st["cache_min"]
    res = {}
    for log2, rows, seed in ((19, 65536, 20250905 + 17), (21, 4 * 65536, 20250905 + 19)):
        tok, lo, hi, ref = bench.rank_pairs(fm, text, bwt, V, seed, dev, rows=rows)
        pc = fm.cache_contains(lo, hi).bool()
        h = torch.clamp(hi, max=n)
        w = torch.where(h > lo, h - lo, torch.zeros_like(lo))
        sym = tok + bench.SHIFT
        live = (w > 0) & (sym >= 0)
        full = live & (lo == 0) & (h == n)
        step = live & ~full
        narrow = step & (w <= 64)
        probe = step & ~narrow & (w >= cache_min)
        empty = (ref[1] <= ref[0])
        # a cached range's probe misses when its symbol is absent (or the key was left out: rare)
        miss = probe & (~pc | empty)
        t1 = step & ~narrow & ~probe & (w <= 512)
        t2 = (step & ~narrow & ~probe & (w > 512)) | miss
        m = tok.numel()
        waves = m // 64
        t1w = t1[: waves * 64].view(waves, 64).sum(1).cpu().numpy()
        t2w = t2[: waves * 64].view(waves, 64).sum(1).cpu().numpy()
        tot = t1w + t2w
        e = {"pairs": int(m), "t1_rows": int(t1.sum()), "t2_rows": int(t2.sum()),
             "probe_rows": int(probe.sum()), "probe_miss_rows": int(miss.sum()),
             "waves": int(waves), "tails_per_wave_mean": float(tot.mean()),
             "hist_tails_per_wave": np.bincount(tot, minlength=12)[:12].tolist(),
             "hist_t1_per_wave": np.bincount(t1w, minlength=8)[:8].tolist(),
             "hist_t2_per_wave": np.bincount(t2w, minlength=8)[:8].tolist(),
             "t1_width_quartiles": (np.percentile(w[t1].cpu().numpy(), [25, 50, 75]).tolist()
                                    if int(t1.sum()) else None)}
        res[f"2^{log2}"] = e
        print(json.dumps(e), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
