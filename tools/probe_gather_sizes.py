"""Random-gather rate vs buffer footprint (TLB reach): fm_probe_gather over
one torch buffer of 4 .. 128 GiB, each access shape, cold; loads per lane 8
and 64.  usage: python tools/probe_gather_sizes.py [--sizes 4,16,32,64,128]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx._lib import check, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4,16,32,64,128")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    res = []
    for gib in [int(x) for x in args.sizes.split(",")]:
        buf = torch.empty((gib << 30) // 8, dtype=torch.int64, device=dev)
        buf.fill_(1)
        for mode, (name, lpl, line) in bench.GATHER_MODES.items():
            for loads in (8, 64):
                threads = 256 * 4096
                best = None
                for _ in range(3):
                    flush.add_(1)
                    torch.cuda.synchronize()
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    a.record()
                    check(lib().fm_probe_gather(buf.data_ptr(), buf.numel() * 8, mode, loads, threads,
                                                sink.data_ptr(), stream), "probe")
                    b.record()
                    torch.cuda.synchronize()
                    ms = a.elapsed_time(b)
                    best = ms if best is None else min(best, ms)
                req = threads // lpl * loads
                e = {"GiB": gib, "shape": name, "loads_per_lane": loads, "us": best * 1e3,
                     "G_req_per_s": req / (best * 1e-3) / 1e9, "GBps": req * line / (best * 1e-3) / 1e9}
                res.append(e)
                print(json.dumps(e), flush=True)
        del buf
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
