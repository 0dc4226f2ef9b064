"""Write floor reference: time K graph-captured fills of the B x V uint8 mask
buffer (torch's fill kernel) and of hipMemsetAsync on the same bytes, to put
the decode kernel's all-rows-empty floor (tools/probe_floor.py) in context.
usage: python tools/probe_memset.py"""
import torch

dev = torch.device("cuda", 0)
B, V, K = 256, 128256, 20
for shape in ((B, V), (B * 8, V)):
    mask = torch.empty(shape, dtype=torch.uint8, device=dev)
    for name, fn in (("torch fill_", lambda: mask.fill_(0)), ("zero_", lambda: mask.zero_())):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(K):
                fn()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            g.replay()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / K * 1e3)
        t = sorted(ts)[2]
        nbytes = mask.numel()
        print(f"{name} {shape[0]}x{shape[1]} ({nbytes / 1e6:.1f} MB): {t:.2f} us/launch -> "
              f"{nbytes / (t * 1e-6) / 1e12:.2f} TB/s", flush=True)
