#!/usr/bin/env python
"""distinct_count for arbitrary wide ranges (not suffix-tree nodes, so the
range cache cannot answer them: the wavelet-matrix BFS of k_distinct) on a
C3-shaped index, across library builds: every library in argv runs in its OWN
process (FMIDX_LIB), times fm_distinct_count_batch over B ranges of
log-uniform width 2^12 .. 2^max cold (1 GiB eviction first) and warm, median
of 5, and checks its output against the first library's (saved .npy).

usage: python tools/bench_distinct_wide.py [--tokens 1e9] [--rows 256] lib_a.so [lib_b.so ...]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
    import numpy as np
    import torch

    import bench

    dev = torch.device("cuda", 0)
    fm, text, bwt, _ = bench.build_index(int(args.tokens), args.vocab, 20250905, dev)
    del text, bwt
    torch.cuda.empty_cache()
    n = fm.size()
    rng = np.random.default_rng(3)
    w = np.exp2(rng.uniform(12, args.max_log2, size=args.rows)).astype(np.int64)
    a = rng.integers(0, n - w.max() - 1, size=args.rows).astype(np.int64)
    lo = torch.tensor(a, device=dev)
    hi = torch.tensor(a + w, device=dev)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    syms, counts, k, off = fm.distinct_count_batch(lo, hi)
    torch.cuda.synchronize()
    t = {}
    for mode in ("cold", "warm"):
        ts = []
        for _ in range(5):
            if mode == "cold":
                flush.add_(1)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            fm.distinct_count_batch(lo, hi)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        t[mode + "_us"] = float(np.median(ts))
    kk = k.cpu().numpy()
    o = off.cpu().numpy()
    s = syms.cpu().numpy()
    c = counts.cpu().numpy()
    flat = np.concatenate([np.stack([s[o[i]:o[i] + kk[i]], c[o[i]:o[i] + kk[i]]], 1) for i in range(args.rows)])
    ref = os.path.join(args.out, "distinct_wide_ref.npz")
    same = None
    if os.path.exists(ref):
        r = np.load(ref)
        same = bool(np.array_equal(r["k"], kk) and np.array_equal(r["flat"], flat))
    else:
        np.savez(ref, k=kk, flat=flat)
    st = {}
    try:
        st = fm.stats()
    except AttributeError:
        pass
    print(json.dumps({"lib": os.path.basename(os.environ.get("FMIDX_LIB", "")), "rows": args.rows,
                      "width_log2": [12, args.max_log2], "cached_rows": int(fm.cache_contains(lo, hi).sum().item()),
                      "symbols_total": int(kk.sum()), **t, "equal_first_lib": same,
                      "device_gib": st.get("device_bytes", 0) / 2**30}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=1e9)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--max-log2", type=int, default=24)
    ap.add_argument("--out", default="/tmp/distinct_wide")   # reference output (large): box-local
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    args = ap.parse_args()
    if args.child:
        child(args)
        return
    os.makedirs(args.out, exist_ok=True)
    ref = os.path.join(args.out, "distinct_wide_ref.npz")
    if os.path.exists(ref):
        os.remove(ref)
    rc = 0
    for lib in args.libs:
        env = dict(os.environ, FMIDX_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--tokens", str(args.tokens),
                            "--vocab", str(args.vocab), "--rows", str(args.rows), "--max-log2", str(args.max_log2),
                            "--out", args.out], env=env)
        rc = rc or r.returncode
        if r.returncode:
            break
    sys.exit(rc)


if __name__ == "__main__":
    main()
