"""Calibration of the PMC fetch counters on random-line gathers (GPU box).

MI355X_MICROARCH.md ("HBM"): FETCH_SIZE reads half the bytes of a wide
coalesced streaming read on gfx950, and "other access widths are
uncalibrated: calibrate on a known byte count in your own access pattern".
The LF kernels read random 8-B words and random 64-B lines, so this runs the
probe kernels of csrc/probe.hip (fm_probe_gather) with a KNOWN number of
independent random lines per dispatch, over an 8 GiB buffer (far past the
256 MiB MALL), one dispatch per access shape in GATHER_MODES order, and
writes the line counts so tools/pmc_calib.sh can divide the counters by them.

usage (under rocprofv3 --pmc ...): python tools/pmc_gather_calib.py --out calib.json
"""
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
    ap.add_argument("--gib", type=int, default=8)
    ap.add_argument("--loads", type=int, default=16)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    nbytes = args.gib << 30
    buf = torch.randint(0, 1 << 62, (nbytes // 8,), dtype=torch.int64, device=dev)
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    threads = 256 * 4096
    order = []
    for mode, (name, lpl, line) in bench.GATHER_MODES.items():
        check(lib().fm_probe_gather(buf.data_ptr(), nbytes, mode, args.loads, threads, sink.data_ptr(), stream),
              "probe")
        torch.cuda.synchronize()
        order.append({"mode": name, "lanes_per_line": lpl, "line_bytes": line,
                      "lines": threads // lpl * args.loads, "line_bytes_total": threads // lpl * args.loads * line})
    json.dump({"buffer_bytes": nbytes, "dispatches": order}, open(args.out, "w"), indent=1)
    print(json.dumps(order))


if __name__ == "__main__":
    main()
