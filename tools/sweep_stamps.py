"""Where a cold 2^19-pair LF launch (the in-wave sweep) spends its time, per wave.

Loads the diagnostic library (libfmidx_stamps.so, built by `make stamps` from
query.hip with profiles/r05_sweep_stamps/sweep_stamps.diff applied), runs the
bench's 2^19 (state, token) pairs in one launch after the bench's clean 1 GiB
eviction, and reads 16 words per wave: stamps (s_memrealtime, 10 ns) at entry,
state used, head loop done (packed E scan of <= 64-row ranges + probes),
tail E scan done, descents done, stores issued; then the head loop's round
trips, the tail scan's, the descent rounds and the wave's probe / tail-scan /
descent / probe-miss row counts.  Prints the launch span, when waves start,
and the phase split of all waves and of the slowest 1 % / 10 %.
usage: python tools/sweep_stamps.py [--tokens 4.5e9] [--reps 3] [--rows-log2 19] [--out f.json]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "fm-index-constrained-decoding_amd")
os.environ["FMIDX_LIB"] = os.path.join(PKG, "fmidx", os.environ.get("STAMPS_LIB", "libfmidx_stamps.so"))
sys.path[:0] = [REPO, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx._lib import lib  # noqa: E402

PH = ["state", "head", "tail_scan", "descents", "stores"]
CN = ["head_rt", "tail_rt", "quad_rounds", "probes", "tail_scan_rows", "descents", "probe_miss"]


def summarize(st, tick_ns=10.0):
    t = st[:, :6].astype(np.int64)
    c = st[:, 6:13].astype(np.int64)
    ok = t[:, 0] > 0
    t, c = t[ok], c[ok]
    t0 = t[:, 0].min()
    rel = (t - t0) * tick_ns / 1e3   # us from the first wave's entry
    span = rel[:, 5] - rel[:, 0]
    ph = np.diff(rel, axis=1)        # 5 phases
    order = np.argsort(span)
    res = {"waves": int(ok.sum()), "launch_span_us": float(rel[:, 5].max()),
           "wave_start_us": {"p50": float(np.median(rel[:, 0])), "p90": float(np.percentile(rel[:, 0], 90)),
                             "max": float(rel[:, 0].max())},
           "wave_end_us": {"p50": float(np.median(rel[:, 5])), "p90": float(np.percentile(rel[:, 5], 90)),
                           "p99": float(np.percentile(rel[:, 5], 99)), "max": float(rel[:, 5].max())},
           "wave_life_us": {"p50": float(np.median(span)), "p90": float(np.percentile(span, 90)),
                            "p99": float(np.percentile(span, 99)), "max": float(span.max())}}
    for name, sel in (("all", order), ("slowest_10pct", order[-max(1, len(order) // 10):]),
                      ("slowest_1pct", order[-max(1, len(order) // 100):])):
        res[name] = {"phase_us": {p: float(ph[sel, k].mean()) for k, p in enumerate(PH)},
                     "counts": {n: float(c[sel, k].mean()) for k, n in enumerate(CN)}}
    # the wave's life against its descent rounds and head-loop round trips
    res["life_by_quad_rounds"] = {int(q): {"waves": int((c[:, 2] == q).sum()), "life_us": float(span[c[:, 2] == q].mean())}
                                  for q in np.unique(c[:, 2])}
    res["life_by_head_rt"] = {int(q): {"waves": int((c[:, 0] == q).sum()), "life_us": float(span[c[:, 0] == q].mean())}
                              for q in np.unique(c[:, 0])}
    # the waves that end last: do they start late (a second round of residency) or live long?
    last = order[-max(1, len(order) // 100):]
    late = np.argsort(rel[:, 5])[-max(1, len(order) // 100):]
    res["last_ending_1pct"] = {"start_us": float(rel[late, 0].mean()), "life_us": float(span[late].mean()),
                               "phase_us": {p: float(ph[late, k].mean()) for k, p in enumerate(PH)},
                               "counts": {n: float(c[late, k].mean()) for k, n in enumerate(CN)}}
    del last
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rows-log2", type=int, default=19)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V = 128256
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    seed = {19: 20250905 + 17, 21: 20250905 + 19}.get(args.rows_log2, 20250905 + 100 + args.rows_log2)
    tok, lo, hi, ref = bench.rank_pairs(fm, text, bwt, V, seed, dev, rows=(1 << args.rows_log2) // 8)
    del text
    torch.cuda.empty_cache()
    m = tok.numel()
    waves = (m + 255) // 256 * 4
    stamps = torch.zeros(waves * 16, dtype=torch.int64, device=dev)
    dl = lib()
    dl.fm_debug_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    acc = torch.zeros((), dtype=torch.int64, device=dev)
    olo, ohi = torch.empty_like(lo), torch.empty_like(hi)
    fm.lf_step_batch(tok, lo, hi, bench.SHIFT, lo_out=olo, hi_out=ohi, reset_below=0)   # code load
    torch.cuda.synchronize()
    out = {"pairs": int(m), "tokens": int(args.tokens), "launches": []}
    for temp in ["cold"] * args.reps + ["warm"]:
        stamps.zero_()
        if temp == "cold":
            flush.add_(1)
            torch.sum(flush, 0, dtype=torch.int64, out=acc)
        torch.cuda.synchronize()
        dl.fm_debug_set_stamps(fm._h, ctypes.c_void_p(stamps.data_ptr()))
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fm.lf_step_batch(tok, lo, hi, bench.SHIFT, lo_out=olo, hi_out=ohi, reset_below=0)
        b.record()
        torch.cuda.synchronize()
        dl.fm_debug_set_stamps(fm._h, None)
        r = summarize(stamps.view(waves, 16).cpu().numpy())
        r["temp"] = temp
        r["event_us"] = a.elapsed_time(b) * 1e3
        r["exact"] = bool(torch.equal(olo, ref[0]) and torch.equal(ohi, ref[1]))
        out["launches"].append(r)
        print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
