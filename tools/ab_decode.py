"""A/B of the fused decode step (the bench's headline kernel) across library
builds: every library in argv runs in its OWN process (FMIDX_LIB), builds the
bench's C3 index (or --tokens), replays the bench's K = 20 trace steps in one
HIP graph cold (after a 1 GiB eviction) and warm, R times each, checks the
final states against the trace and every step's mask against the first
library's (saved masks), and prints one JSON line per library.

usage: python tools/ab_decode.py [--tokens 4.5e9] [--reps 7] lib_a.so lib_b.so ...
A library argument may carry build options for its process:
lib.so@trans_min=2,lf_e=0 (FMIDX_BUILD_OPTIONS); the line then reports the
index's device bytes and transition-table counts too.  A %-suffix sets the
process's FMIDX_TUNING: lib.so%dec_threads=512 (or lib.so@opts%tuning).
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
    from fmidx.synth import decode_trace

    dev = torch.device("cuda", 0)
    V, B, K, W, SHIFT = 128256, args.batch, 20, 5, 10
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    tokens, init, lo_hist, hi_hist, _ = decode_trace(fm, text, bwt, B, V, W + K, 20250905, dev)
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
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)

    def timed(cold):
        lo.copy_(st_lo)
        hi.copy_(st_hi)
        if cold:
            flush.add_(1)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / K

    timed(False)
    cold = [timed(True) for _ in range(args.reps)]
    warm = [timed(False) for _ in range(args.reps)]
    fin = bufs[K % 2]
    ok = bool(torch.equal(fin[0], lo_hist[W + K - 1]) and torch.equal(fin[1], hi_hist[W + K - 1]))
    # the last step's mask against the first library's
    ref = os.path.join(args.out, "ab_mask.npy")
    m = mask.cpu().numpy()
    same = None
    if os.path.exists(ref):
        same = bool(np.array_equal(np.load(ref), m))
    else:
        np.save(ref, m)
    try:
        st = fm.stats()
    except AttributeError:     # a library older than the stats it asks for
        st = {"device_bytes": 0, "trans_bytes": 0, "trans_entries": -1, "trans_dropped": -1}
    print(json.dumps({"lib": os.environ.get("FMIDX_LIB"), "build_options": os.environ.get("FMIDX_BUILD_OPTIONS", ""), "tuning": os.environ.get("FMIDX_TUNING", ""),
                      "device_gib": st["device_bytes"] / 2**30, "trans_gib": st["trans_bytes"] / 2**30,
                      "trans_entries": st["trans_entries"], "trans_dropped": st["trans_dropped"], "cold_us": sorted(cold), "warm_us": sorted(warm),
                      "cold_median": float(np.median(cold)), "warm_median": float(np.median(warm)),
                      "trace_ok": ok, "mask_equal_first_lib": same}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default="/tmp/ab_decode")   # the saved mask: box-local
    ap.add_argument("--child", action="store_true")
    ap.add_argument("libs", nargs="*")
    args = ap.parse_args()
    if args.child:
        child(args)
        return
    os.makedirs(args.out, exist_ok=True)
    ref = os.path.join(args.out, "ab_mask.npy")
    if os.path.exists(ref):
        os.remove(ref)
    rc = 0
    for lib in args.libs:
        lib, _, tun = lib.partition("%")
        lib, _, opts = lib.partition("@")
        env = dict(os.environ, FMIDX_LIB=os.path.abspath(lib))
        if opts:
            env["FMIDX_BUILD_OPTIONS"] = opts
        if tun:
            env["FMIDX_TUNING"] = tun
        r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "--child", "--tokens", str(args.tokens),
                            "--batch", str(args.batch), "--reps", str(args.reps), "--out", args.out], env=env)
        rc = rc or r.returncode
        if r.returncode:
            break
    sys.exit(rc)


if __name__ == "__main__":
    main()
