"""distinct_count_multi (fm_index.cpp:146-166) on the C3-scale
index: the call the reference's processors make every decode step
(get_distinct_count_multi over the B rows' ranges, index.py:161-174).

For B = 256 rows of the bench's decode trace at several steps: the device
launch alone (fm_distinct_count_batch: cached ranges from their bitmaps and
the transition table, the rest by the 2-level wavelet-matrix BFS, one workgroup
per range), and the SWIG-surface call end to end (fm_distinct_count_multi: launch +
device compaction + copy + Python tuples), against oracle/cpu_ref's
sdsl-faithful distinct_count (the reference's algorithm, sigma-sized scratch per
call) on one thread and on all cores.  Results must agree exactly.

usage: python tools/bench_distinct.py [--tokens 4.5e9] [--steps 6]
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx.synth import decode_trace  # noqa: E402
from oracle.cpu_ref import CpuRef  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    V = 128256
    fm, text, bwt, _ = bench.build_index(int(args.tokens), V, 20250905, dev)
    n = bwt.numel()
    B, S = args.batch, args.steps
    tokens, _, lo_h, hi_h, _ = decode_trace(fm, text, bwt, B, V, S, 99, dev)
    del text
    ref = CpuRef.from_device_bwt(bwt)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    res = {"corpus_tokens": n, "batch": B, "steps": []}
    cores = len(os.sched_getaffinity(0))
    pool = ThreadPoolExecutor(max_workers=cores)
    for s in range(S):
        lo, hi = lo_h[s].contiguous(), hi_h[s].contiguous()
        w = (hi - lo).cpu().numpy()

        def dev_call():
            return fm.distinct_count_batch(lo, hi)

        times = {}
        for mode in ("cold", "warm"):
            best = None
            for _ in range(3):
                if mode == "cold":
                    flush.add_(1)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                out = dev_call()
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b)
                best = ms if best is None else min(best, ms)
            times[mode] = best * 1e3
        syms, counts, k, cap_off = out
        lows = lo.cpu().numpy().astype(np.uint64)
        highs = hi.cpu().numpy().astype(np.uint64)
        t0 = time.perf_counter()
        host = fm.distinct_count_multi(lows.tolist(), highs.tolist())
        host_us = (time.perf_counter() - t0) * 1e6
        t0 = time.perf_counter()
        cpu1 = [ref.distinct_count(int(a), int(b)) for a, b in zip(lows, highs)]
        cpu1_us = (time.perf_counter() - t0) * 1e6
        t0 = time.perf_counter()
        cpun = list(pool.map(lambda ab: ref.distinct_count(int(ab[0]), int(ab[1])), zip(lows, highs)))
        cpun_us = (time.perf_counter() - t0) * 1e6
        ok = tuple(tuple(x) for x in cpu1) == host and cpun == cpu1
        kk = k.cpu().numpy()
        co = cap_off.cpu().numpy()
        sy = syms.cpu().numpy()
        ct = counts.cpu().numpy()
        dev_ok = all(tuple(int(v) for pair in zip(sy[co[i]:co[i] + kk[i]], ct[co[i]:co[i] + kk[i]]) for v in pair)
                     == tuple(cpu1[i]) for i in range(B))
        e = {"step": s, "device_cold_us": times["cold"], "device_warm_us": times["warm"],
             "host_api_us": host_us, "cpu_1thread_us": cpu1_us, f"cpu_{cores}threads_us": cpun_us,
             "symbols_out": int(kk.sum()), "max_width": int(w.max()), "rows_wider_4096": int((w > 4096).sum()),
             "exact": bool(ok and dev_ok)}
        res["steps"].append(e)
        print(f"step {s}: device {times['cold']:.0f} us cold / {times['warm']:.0f} warm, host API {host_us:.0f} us, "
              f"cpu_ref 1 thread {cpu1_us:.0f} us, {cores} threads {cpun_us:.0f} us; {int(kk.sum())} symbols, "
              f"{int((w > 4096).sum())} rows > 4096 wide (max {int(w.max())}); exact {e['exact']}", flush=True)
    res["cores"] = cores
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
