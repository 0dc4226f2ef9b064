"""The batching query service (fmidx/service.py) against the reference's
service routes (fm_index_api_service.py:101-255): every route's response equals
the index's own answer, concurrent requests are answered by fewer batched
searches than requests, and a bad pattern fails only its own request.  The CPU
tests run the service over the oracle index (duck-typed, test-only); the GPU
test over the product FMIndex."""
import asyncio
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]

httpx = pytest.importorskip("httpx")
pytest.importorskip("fastapi")

from fmidx.service import create_app  # noqa: E402


def _corpus(seed=5, n_docs=40, vocab=30):
    rng = np.random.default_rng(seed)
    return [rng.integers(0, vocab, size=int(rng.integers(3, 40))).tolist() for _ in range(n_docs)]


class _OracleAdapter:
    """OracleIndex plus the batched search the service calls."""

    def __init__(self, docs):
        from oracle.fm_oracle import OracleIndex

        self.ix = OracleIndex()
        self.ix.initialize(docs)

    def __getattr__(self, name):
        return getattr(self.ix, name)

    def __len__(self):
        return len(self.ix)

    def get_ranges(self, seqs):
        return [self.ix.get_range(s) for s in seqs]


def _patterns(docs, rng, k):
    out = []
    for _ in range(k):
        d = docs[int(rng.integers(len(docs)))]
        a = int(rng.integers(len(d)))
        out.append(d[a:a + int(rng.integers(1, 5))] if rng.random() < 0.8 else rng.integers(0, 40, 3).tolist())
    return out


async def _exercise(index, expect):
    """expect: the reference-behaving index the answers must equal."""
    app = create_app(index=index, window_s=2e-3)
    rng = np.random.default_rng(11)
    docs = [expect.get_doc(d) for d in range(expect.n_docs)]
    pats = _patterns(docs, rng, 64)
    async with app.router.lifespan_context(app):
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            h = (await c.get("/health")).json()
            assert h == {"status": "healthy", "n_docs": expect.n_docs, "n_tokens": len(expect)}
            # concurrent single-pattern requests -> fewer batched searches
            rs = await asyncio.gather(*[c.post("/get_count", json={"sub_sequence": p}) for p in pats])
            assert [r.json()["count"] for r in rs] == [expect.get_count(p) for p in pats]
            st = (await c.get("/stats")).json()
            assert st["patterns"] >= len(pats) and st["batches"] < len(pats) and st["largest_batch"] > 1
            rs = await asyncio.gather(*[c.post("/get_range", json={"sequence": p}) for p in pats[:16]])
            assert [tuple(r.json()["range"]) for r in rs] == [expect.get_range(p) for p in pats[:16]]
            rs = await asyncio.gather(*[c.post("/continuations", json={"sequence": p}) for p in pats[:16]])
            assert [r.json()["continuations"] for r in rs] == [expect.get_continuations(p) for p in pats[:16]]
            for p in pats[:6] + [[]]:
                r = (await c.post("/search", json={"sequence": p, "limit": 5})).json()
                assert r["count"] == expect.get_count(p)
                assert r["doc_indices"] == list(expect.get_doc_indices(p))[:5]
            lows = [expect.get_range(p)[0] for p in pats[:8]]
            highs = [expect.get_range(p)[1] for p in pats[:8]]
            r = (await c.post("/get_distinct_count_multi", json={"lows": lows, "highs": highs})).json()
            assert [tuple(map(list, x)) for x in r["distinct_list"]] == \
                [tuple(map(list, x)) for x in expect.get_distinct_count_multi(lows, highs)]
            r = (await c.get("/docs/3")).json()
            assert r["tokens"] == expect.get_doc(3) and r["length"] == len(expect.get_doc(3))
            assert (await c.get(f"/docs/{expect.n_docs}")).status_code == 404
            assert (await c.get("/occurring_distinct")).json() == list(expect.occurring_distinct)
            # batched routes
            r = (await c.post("/get_count_batch", json={"sequences": pats})).json()
            assert r["counts"] == [expect.get_count(p) for p in pats]
            r = (await c.post("/get_range_batch", json={"sequences": pats[:10]})).json()
            assert [tuple(x) for x in r["ranges"]] == [expect.get_range(p) for p in pats[:10]]
            r = (await c.post("/continuations_batch", json={"sequences": pats[:10]})).json()
            assert r["continuations"] == [expect.get_continuations(p) for p in pats[:10]]
            # a pattern below the symbol range fails alone (500), its batch-mates succeed
            bad, good = await asyncio.gather(c.post("/get_count", json={"sub_sequence": [1, -20]}),
                                             c.post("/get_count", json={"sub_sequence": pats[0]}))
            assert bad.status_code == 500 and good.json()["count"] == expect.get_count(pats[0])


def test_service_routes_over_oracle():
    ix = _OracleAdapter(_corpus())
    asyncio.run(_exercise(ix, ix.ix))


@pytest.mark.gpu
def test_service_routes_on_gpu():
    from fmidx.index import FMIndex
    from oracle.fm_oracle import OracleIndex

    docs = _corpus(seed=9, n_docs=60)
    ix = FMIndex(device=0)
    ix.initialize(docs)
    ref = OracleIndex()
    ref.initialize(docs)
    asyncio.run(_exercise(ix, ref))
