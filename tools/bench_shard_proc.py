#!/usr/bin/env python
"""A logits-processor call over a doc-range sharded index (fmidx.sharding.
ShardedIndex) against the same call on the unsharded index, on
one GPU through RCCL at world 1 (the whole corpus as the only shard): what the
sharded machinery itself costs -- fm_processor_shard_prep, the facts
all_reduce, the allowed-bits exchange (sparse all_gather, peer with the RCCL
barrier, peer with the flag barrier), fm_processor_shard_finish -- next to the
one-call fused path.  Qwen processor, B = 256 rows (128 x 2 beams), bf16
scores over 151936 tokens, an index of --tokens tokens; every call checked
against the unsharded output.  Medians of --calls calls (host wall, each
call's output synchronised).

usage: python tools/bench_shard_proc.py [--tokens 1e9] [--calls 30]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=1e9)
    ap.add_argument("--calls", type=int, default=30)
    args = ap.parse_args()
    import torch.distributed as dist

    import fmidx.processors as P
    from fmidx.sharding import ShardedIndex

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    V = 151936
    fm, text, bwt, _ = bench.build_index(int(args.tokens), 128256, 20250905, dev)
    del bwt
    n = text.numel()
    raw = fm.distinct_count(0, n - 1)
    fm.occurring_distinct = [s - 10 for s in raw[0::2] if s > 0]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{bench.free_port()}", world_size=1, rank=0,
                            device_id=dev)
    rng = np.random.default_rng(3)
    beams, groups = 2, 128
    B = beams * groups
    q = rng.integers(0, n - 64, size=B)
    head = [151644, 872, 198, 151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]
    body = [[int(text[(n - 2) - (int(a) + k)].item()) - 10 for k in range(6)] for a in q]
    kw = dict(num_beams=beams, pad_token_id=151643, eos_token_id=151645, min_new_tokens=1, length_reward_factor=1.0)
    ref = P.QwenIndexBasedLogitsProcessor(index=fm, **kw)
    res = {"n": n, "rows": B, "vocab": V, "calls": args.calls}
    variants = {"unsharded": ref}
    sidx = {}
    for name, ex, pb in (("sparse", "sparse", "collective"), ("peer", "peer", "collective"),
                         ("peer_flags", "peer", "flags")):
        sidx[name] = ShardedIndex(fm, fm.occurring_distinct, group=dist.group.WORLD, exchange=ex, peer_barrier=pb)
        variants[name] = P.QwenIndexBasedLogitsProcessor(index=sidx[name], **kw)
    times = {k: [] for k in variants}
    exact = {k: True for k in variants}
    for c in range(args.calls + 3):
        ids = torch.tensor([head + b + [int(x) for x in rng.integers(100, 5000, size=c % 4)] for b in body],
                           dtype=torch.int64, device=dev)
        scores = torch.from_numpy(rng.standard_normal((B, V)).astype(np.float32)).to(torch.bfloat16).to(dev)
        want = None
        for k, proc in variants.items():
            x = scores.clone()
            torch.cuda.synchronize()
            a = time.perf_counter()
            out = proc(ids, x)
            torch.cuda.synchronize()
            t = time.perf_counter() - a
            if c >= 3:
                times[k].append(t)
            if want is None:
                want = out.clone()
            elif not torch.equal(out.view(torch.int16), want.view(torch.int16)):
                exact[k] = False
    for k in variants:
        res[k] = {"ms_per_call_median": float(np.median(times[k])) * 1e3, "equal_unsharded": exact[k]}
        print(f"{k:12s} {res[k]['ms_per_call_median']:.3f} ms/call, exact {exact[k]}", file=sys.stderr, flush=True)
    for s in sidx.values():
        s.close()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
