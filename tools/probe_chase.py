"""Dependent random 64-B hops (csrc/probe.hip k_chase64, 256 chains) over
buffers of growing size, each pass after a 1 GiB cache eviction: how much of
a cold round trip is the page-table walk (TLB reach) rather than HBM."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import torch  # noqa: E402

from fmidx._lib import check, lib  # noqa: E402

dev = torch.device("cuda", 0)
flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
sink = torch.zeros(1024, dtype=torch.int64, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
for gb in (0.0625, 0.25, 1, 4, 16, 64, 160):
    nbytes = int(gb * (1 << 30))
    buf = torch.randint(0, 1 << 62, (nbytes // 8,), dtype=torch.int64, device=dev)
    for chains, hops in ((256, 2000), (16384, 500)):
        flush.add_(1)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        check(lib().fm_probe_gather(buf.data_ptr(), nbytes, 1, hops, chains, sink.data_ptr(), stream), "chase")
        b.record()
        torch.cuda.synchronize()
        ns = a.elapsed_time(b) * 1e6 / hops
        print(f"buffer {gb:8.4f} GiB  chains {chains:6d}: {ns:7.0f} ns/hop  "
              f"({chains * 64 / ns:8.1f} GB/s of 64-B lines)", flush=True)
    del buf
    torch.cuda.empty_cache()
