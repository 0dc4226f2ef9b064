"""Query-service throughput (fmidx/service.py) on a device-built index:
/get_count requests with C clients in flight (in-process ASGI transport, so
the HTTP stack's serialization is measured but no sockets), the batched route,
the same service with batching off (one search per request, the reference's
serving model, fm_index_api_service.py:147-161), and `get_count` called once
per pattern without HTTP.
Usage: python tools/bench_service.py [--tokens N] [--requests R] [--clients C]"""
import argparse
import asyncio
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import httpx  # noqa: E402

from fmidx.fm_index import suffix_sort_device  # noqa: E402
from fmidx.index import FMIndex  # noqa: E402
from fmidx.service import create_app  # noqa: E402
from fmidx.synth import markov_corpus_gpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=float, default=1e9)
ap.add_argument("--vocab", type=int, default=128256)
ap.add_argument("--requests", type=int, default=4096)
ap.add_argument("--clients", type=int, default=256)
ap.add_argument("--serial", type=int, default=512)
args = ap.parse_args()
dev = torch.device("cuda", 0)
SHIFT = 10

t0 = time.perf_counter()
text, beg = markov_corpus_gpu(int(args.tokens), args.vocab, 20250905, dev)
bwt, _ = suffix_sort_device(text)
ix = FMIndex(device=0)
ix.initialize_from_bwt_device(bwt)
ix.beginnings = beg.cpu().tolist()
ix.occurring_distinct, ix.occurring_counts = ix.get_distinct_count(0, len(ix))
build_s = time.perf_counter() - t0
n = text.numel()
g = torch.Generator(device=dev)
g.manual_seed(4)
R = args.requests
q = torch.randint(0, n - 64, (R,), generator=g, device=dev)
L = torch.randint(1, 9, (R,), generator=g, device=dev)
win = text[q[:, None] + torch.arange(8, device=dev)[None, :]].to(torch.int64).cpu().numpy() - SHIFT
lens = L.cpu().numpy()
# F is reverse(T'): a substring of T' read backwards is a pattern of the corpus
pats = [[int(x) for x in win[i, : lens[i]][::-1]] for i in range(R)]
del text, bwt
torch.cuda.empty_cache()
truth = [hi - lo for lo, hi in ix.get_ranges(pats)]

# serial: one blocking search per request
t = time.perf_counter()
ser = [ix.get_count(p) for p in pats[: args.serial]]
serial_s = time.perf_counter() - t
assert ser == truth[: args.serial]


async def run(batching):
    app = create_app(index=ix, window_s=2e-4, batching=batching)
    async with app.router.lifespan_context(app):
        tr = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=tr, base_url="http://t") as c:
            sem = asyncio.Semaphore(args.clients)
            got = [None] * R

            async def one(i):
                async with sem:
                    r = await c.post("/get_count", json={"sub_sequence": pats[i]})
                    got[i] = r.json()["count"]

            await asyncio.gather(*[one(i) for i in range(min(R, 512))])   # warm
            st0 = (await c.get("/stats")).json()
            t1 = time.perf_counter()
            await asyncio.gather(*[one(i) for i in range(R)])
            conc_s = time.perf_counter() - t1
            st1 = (await c.get("/stats")).json()
            assert got == truth
            t2 = time.perf_counter()
            r = (await c.post("/get_count_batch", json={"sequences": pats})).json()
            batch_s = time.perf_counter() - t2
            assert r["counts"] == truth
            return conc_s, batch_s, st1["batches"] - st0["batches"], st1["largest_batch"]


conc_s, batch_s, nb, largest = asyncio.run(run(True))
conc1_s, _, nb1, _ = asyncio.run(run(False))
res = {"corpus_tokens": n, "index_build_s": round(build_s, 1), "requests": R, "clients": args.clients,
       "serial_get_count": {"calls": args.serial, "us_per_call": round(serial_s / args.serial * 1e6, 1),
                            "req_per_s": round(args.serial / serial_s)},
       "service_get_count": {"req_per_s": round(R / conc_s), "batches": nb, "mean_batch": round(R / max(nb, 1), 1),
                             "largest_batch": largest},
       "service_get_count_unbatched": {"req_per_s": round(R / conc1_s), "searches": nb1},
       "service_get_count_batch": {"patterns_per_s": round(R / batch_s), "ms": round(batch_s * 1e3, 2)}}
print(json.dumps(res), flush=True)
