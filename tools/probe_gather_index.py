"""Random-gather rate over the index's OWN allocations (fm_device_struct) vs a
buffer allocated after the build, at C3 scale: is the rank kernels' read rate
set by where the structures live (page fragmentation / TLB) rather than by
the access shape?  usage: python tools/probe_gather_index.py [--tokens 4.5e9]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx._lib import check, lib  # noqa: E402

NAMES = {0: "bwt", 1: "E", 2: "trans", 3: "cache_bm", 4: "w2_level0"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--fresh-gib", type=int, default=32)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    fm, text, bwt, _ = bench.build_index(int(args.tokens), 128256, 20250905, dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)

    def rate(ptr, nbytes, mode, loads):
        name, lpl, line = bench.GATHER_MODES[mode]
        threads = 256 * 4096
        best = None
        for _ in range(3):
            flush.add_(1)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            check(lib().fm_probe_gather(ptr, nbytes, mode, loads, threads, sink.data_ptr(), stream), "probe")
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        return threads // lpl * loads / (best * 1e-3) / 1e9

    targets = [(NAMES[w],) + fm.device_struct(w) for w in NAMES]
    del text
    torch.cuda.empty_cache()
    fresh = torch.empty((args.fresh_gib << 30) // 8, dtype=torch.int64, device=dev)
    fresh.fill_(1)
    targets.append((f"fresh_{args.fresh_gib}GiB_after_build", fresh.data_ptr(), fresh.numel() * 8))
    res = []
    for name, ptr, nbytes in targets:
        if not ptr or nbytes < (1 << 20):
            continue
        for mode in (4, 2):
            for loads in (8, 64):
                g = rate(ptr, nbytes, mode, loads)
                e = {"target": name, "GiB": nbytes / 2**30, "shape": bench.GATHER_MODES[mode][0], "loads": loads,
                     "G_req_per_s": g}
                res.append(e)
                print(json.dumps(e), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
