"""Random-access THROUGHPUT against the size of the region (TLB reach): the
gather probe (csrc/probe.hip) over torch buffers of growing size, for
every-lane-its-own-8-B-word (an LF step's E read) and 4-lanes-per-64-B-line
shapes.  Complements tools/micro/tlb.hip (latency per dependent hop).

usage: python tools/probe_tlb_rate.py [--sizes-gib 4,16,32,64,128]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

from fmidx._lib import check, lib  # noqa: E402

MODES = {4: ("lane_8B", 1, 8), 2: ("coop4_64B", 4, 64), 3: ("coop8_128B", 8, 128)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-gib", default="4,16,32,64,128")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    out = {}
    for g in [int(x) for x in args.sizes_gib.split(",")]:
        nbytes = g << 30
        buf = torch.empty(nbytes // 8, dtype=torch.int64, device=dev)
        buf[:: 1 << 20] = 1
        res = {}
        for mode, (name, lpl, line) in MODES.items():
            best = None
            for _ in range(3):
                flush.add_(1)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                check(lib().fm_probe_gather(buf.data_ptr(), nbytes, mode, 64, 256 * 4096, sink.data_ptr(), stream),
                      "probe")
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b)
                best = ms if best is None else min(best, ms)
            res[name] = {"GBps": 256 * 4096 // lpl * 64 * line / (best * 1e-3) / 1e9,
                         "G_lines_per_s": 256 * 4096 // lpl * 64 / (best * 1e-3) / 1e9}
        out[f"{g}GiB"] = res
        print(g, "GiB", {k: round(v["G_lines_per_s"], 1) for k, v in res.items()}, "G lines/s", flush=True)
        del buf
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
