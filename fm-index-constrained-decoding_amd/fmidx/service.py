"""The index query service with request batching.

Same routes, request and response models as the reference's FastAPI service
(fm_index_api_service.py:26-65 models, :101-255 routes): /health, /search,
/occurring_distinct, /get_count, /get_range, /get_distinct_count_multi,
/continuations, /docs/{doc_index}, /stats, with `took_ms` in the responses and
503 / 404 / 500 as there.  The difference is how requests reach the index.
The reference's handlers are `async def` functions that make blocking calls,
so requests serialize on the event loop, one backward search each.  Here the
pattern searches of all requests in flight are collected by a micro-batcher
and answered by ONE batched search (fm_get_range_batch, one wave per
pattern), run on a single worker thread, so the event loop keeps accepting
requests while the GPU works.  The continuations of a batch are one batched
distinct-count launch as well.  Batched routes (/get_count_batch,
/get_range_batch, /continuations_batch) take many patterns in one request.

The index is any object with the reference FMIndex's query methods plus
`get_ranges(list of patterns)`; `fmidx.index.FMIndex` is the product one.
Run: FM_INDEX_PATH=<path> python -m fmidx.service [--port 8000]
"""
import asyncio
import itertools
import logging
import os
import time
from concurrent.futures import ThreadPoolExecutor
from contextlib import asynccontextmanager
from typing import List, Optional, Tuple

from fastapi import FastAPI, HTTPException
from pydantic import BaseModel

logger = logging.getLogger(__name__)
SHIFT = 10   # index.py:16


# -- request / response models (fm_index_api_service.py:26-65) -------------
class SearchRequest(BaseModel):
    sequence: List[int]
    limit: Optional[int] = 100


class SearchResponse(BaseModel):
    count: int
    doc_indices: List[int]
    took_ms: float


class ContinuationRequest(BaseModel):
    sequence: List[int]


class ContinuationResponse(BaseModel):
    continuations: List[int]
    took_ms: float


class CountRequest(BaseModel):
    sub_sequence: List[int]


class CountResponse(BaseModel):
    count: int
    took_ms: float


class RangeRequest(BaseModel):
    sequence: List[int]


class RangeResponse(BaseModel):
    range: Tuple[int, int]
    took_ms: float


class DistinctRequest(BaseModel):
    lows: List[int]
    highs: List[int]


class DistinctResponse(BaseModel):
    distinct_list: List[Tuple[List[int], List[int]]]
    took_ms: float


# -- batched routes ----------------------------------------------------------
class BatchRequest(BaseModel):
    sequences: List[List[int]]


class BatchCountResponse(BaseModel):
    counts: List[int]
    took_ms: float


class BatchRangeResponse(BaseModel):
    ranges: List[Tuple[int, int]]
    took_ms: float


class BatchContinuationResponse(BaseModel):
    continuations: List[List[int]]
    took_ms: float


class RangeBatcher:
    """Collects the patterns of concurrent requests and resolves them with one
    `index.get_ranges` call per batch.  A batch closes when `max_batch`
    patterns are waiting or `window_s` after its first request arrived; the
    search runs on the (single) index worker thread.  A request's patterns
    (one, or many for the batched routes) share one future."""

    def __init__(self, index, worker: ThreadPoolExecutor, window_s: float = 2e-4, max_batch: int = 4096,
                 batching: bool = True):
        self.index = index
        self.batching = batching   # False: one search per request (the reference's serving model)
        self.worker = worker
        self.window_s = window_s
        self.max_batch = max_batch
        self._pending: List[Tuple[List[List[int]], asyncio.Future]] = []
        self._npending = 0
        self._kick: Optional[asyncio.Event] = None
        self._task: Optional[asyncio.Task] = None
        self.batches = 0          # launches issued
        self.patterns = 0         # patterns answered
        self.largest = 0

    def start(self) -> None:
        self._kick = asyncio.Event()
        self._task = asyncio.get_running_loop().create_task(self._run())

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass
            self._task = None
        for _, fut in self._pending:
            if not fut.done():
                fut.set_exception(RuntimeError("service shutting down"))
        self._pending = []
        self._npending = 0

    async def ranges(self, seqs: List[List[int]]) -> List[Tuple[int, int]]:
        # a pattern the reference's backward_search_step rejects (a symbol
        # below 0: SWIG's OverflowError, a 500) fails its own request only
        for s in seqs:
            if s and min(s) + SHIFT < 0:
                raise OverflowError("in method 'FMIndex_backward_search_step', argument 2 of type 'char_type'")
        if not seqs:
            return []
        if not self.batching:
            res = await asyncio.get_running_loop().run_in_executor(self.worker, self.index.get_ranges, seqs)
            self.batches += 1
            self.patterns += len(seqs)
            self.largest = max(self.largest, len(seqs))
            return [(int(lo), int(hi)) for lo, hi in res]
        fut = asyncio.get_running_loop().create_future()
        self._pending.append((seqs, fut))
        self._npending += len(seqs)
        self._kick.set()
        return await fut

    async def _run(self) -> None:
        loop = asyncio.get_running_loop()
        while True:
            await self._kick.wait()
            self._kick.clear()
            if not self._pending:
                continue
            # let the requests that are already on their way join this batch
            t_end = loop.time() + self.window_s
            while self._npending < self.max_batch and loop.time() < t_end:
                await asyncio.sleep(0)
            batch, n = [], 0
            while self._pending and (not batch or n + len(self._pending[0][0]) <= self.max_batch):
                req = self._pending.pop(0)
                batch.append(req)
                n += len(req[0])
            self._npending -= n
            if self._pending:
                self._kick.set()
            seqs = [s for req, _ in batch for s in req]
            try:
                res = await loop.run_in_executor(self.worker, self.index.get_ranges, seqs)
                pos = 0
                for req, fut in batch:
                    part = [(int(lo), int(hi)) for lo, hi in res[pos:pos + len(req)]]
                    pos += len(req)
                    if not fut.done():
                        fut.set_result(part)
            except Exception as e:          # every request of the batch gets the error (500)
                for _, fut in batch:
                    if not fut.done():
                        fut.set_exception(e)
            self.batches += 1
            self.patterns += n
            self.largest = max(self.largest, n)


def create_app(index=None, index_path: Optional[str] = None, window_s: float = 2e-4,
               max_batch: int = 4096, batching: bool = True) -> FastAPI:
    """The service around `index` (or the index saved at `index_path` /
    $FM_INDEX_PATH, loaded at startup as in fm_index_api_service.py:68-90)."""
    state = {"index": index, "batcher": None}
    worker = ThreadPoolExecutor(max_workers=1, thread_name_prefix="fmidx-index")

    @asynccontextmanager
    async def lifespan(app: FastAPI):
        if state["index"] is None:
            from .index import FMIndex

            path = index_path or os.getenv("FM_INDEX_PATH", "data/PAQ/PAQ_index/PAQ.fm_index")
            t0 = time.time()
            state["index"] = await asyncio.get_running_loop().run_in_executor(worker, FMIndex.load, path)
            logger.info("FM-Index loaded from %s in %.2fs", path, time.time() - t0)
        b = RangeBatcher(state["index"], worker, window_s, max_batch, batching)
        b.start()
        state["batcher"] = b
        app.state.batcher = b
        yield
        await b.stop()
        worker.shutdown(wait=True)

    app = FastAPI(title="FM-Index Search Service", version="1.0.0", lifespan=lifespan)

    def ix():
        if state["index"] is None or state["batcher"] is None:
            raise HTTPException(status_code=503, detail="FM-Index not loaded")
        return state["index"]

    async def on_worker(fn, *args):
        return await asyncio.get_running_loop().run_in_executor(worker, fn, *args)

    async def continuations_of(index, ranges):
        lows = [lo for lo, _ in ranges]
        highs = [hi for _, hi in ranges]
        # get_continuations == get_distinct(get_range(seq)) (index.py:131-136):
        # the distinct symbols of every range in one batched launch
        multi = await on_worker(index.get_distinct_count_multi, lows, highs)
        return [list(syms) for syms, _ in multi]

    @app.get("/health")
    async def health_check():
        index = ix()
        return {"status": "healthy", "n_docs": index.n_docs, "n_tokens": len(index)}

    @app.post("/search", response_model=SearchResponse)
    async def search(request: SearchRequest):
        index = ix()
        t0 = time.time()
        try:
            (lo, hi), = await state["batcher"].ranges([request.sequence])
            count = hi - lo
            docs = []
            if count > 0:
                lim = request.limit
                # get_doc_indices yields in row order, located chunk by chunk on the device:
                # with a limit only the chunks that reach it are located (the reference
                # slices the full list, fm_index_api_service.py:121-124 -- same output)
                if lim and lim > 0:
                    docs = await on_worker(lambda: list(itertools.islice(index.get_doc_indices(request.sequence),
                                                                         lim)))
                else:
                    docs = await on_worker(lambda: list(index.get_doc_indices(request.sequence)))
                    if lim and len(docs) > lim:      # a negative limit slices from the end, as there
                        docs = docs[:lim]
            return SearchResponse(count=count, doc_indices=docs, took_ms=(time.time() - t0) * 1000)
        except HTTPException:
            raise
        except Exception as e:
            logger.error("Search error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.get("/occurring_distinct")
    async def get_occurring_distinct():
        return ix().occurring_distinct

    @app.post("/get_count")
    async def get_count(request: CountRequest):
        ix()
        t0 = time.time()
        try:
            (lo, hi), = await state["batcher"].ranges([request.sub_sequence])
            return CountResponse(count=hi - lo, took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            logger.error("Get count error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/get_range")
    async def get_range(request: RangeRequest):
        ix()
        t0 = time.time()
        try:
            (lo, hi), = await state["batcher"].ranges([request.sequence])
            return RangeResponse(range=(lo, hi), took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            logger.error("Get range error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/get_distinct_count_multi")
    async def get_distinct_count_multi(request: DistinctRequest):
        index = ix()
        t0 = time.time()
        try:
            dl = await on_worker(index.get_distinct_count_multi, request.lows, request.highs)
            return DistinctResponse(distinct_list=dl, took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            logger.error("Get distinct error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/continuations", response_model=ContinuationResponse)
    async def get_continuations(request: ContinuationRequest):
        index = ix()
        t0 = time.time()
        try:
            r = await state["batcher"].ranges([request.sequence])
            cont, = await continuations_of(index, r)
            return ContinuationResponse(continuations=cont, took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            logger.error("Continuations error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.get("/docs/{doc_index}")
    async def get_document(doc_index: int):
        index = ix()
        if doc_index < 0 or doc_index >= index.n_docs:
            raise HTTPException(status_code=404, detail="Document not found")
        try:
            doc = await on_worker(index.get_doc, doc_index)
            return {"doc_index": doc_index, "tokens": doc, "length": len(doc)}
        except Exception as e:
            logger.error("Document retrieval error: %s", e)
            raise HTTPException(status_code=500, detail=str(e))

    @app.get("/stats")
    async def get_stats():
        index = ix()
        b = state["batcher"]
        return {"n_docs": index.n_docs, "n_tokens": len(index), "occurring_tokens": len(index.occurring),
                "has_labels": index.labels is not None,
                "batches": b.batches, "patterns": b.patterns, "largest_batch": b.largest}

    # -- batched routes --------------------------------------------------------
    @app.post("/get_count_batch", response_model=BatchCountResponse)
    async def get_count_batch(request: BatchRequest):
        ix()
        t0 = time.time()
        try:
            r = await state["batcher"].ranges(request.sequences)
            return BatchCountResponse(counts=[hi - lo for lo, hi in r], took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/get_range_batch", response_model=BatchRangeResponse)
    async def get_range_batch(request: BatchRequest):
        ix()
        t0 = time.time()
        try:
            r = await state["batcher"].ranges(request.sequences)
            return BatchRangeResponse(ranges=r, took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))

    @app.post("/continuations_batch", response_model=BatchContinuationResponse)
    async def continuations_batch(request: BatchRequest):
        index = ix()
        t0 = time.time()
        try:
            r = await state["batcher"].ranges(request.sequences)
            cont = await continuations_of(index, r)
            return BatchContinuationResponse(continuations=cont, took_ms=(time.time() - t0) * 1000)
        except Exception as e:
            raise HTTPException(status_code=500, detail=str(e))

    return app


def main() -> None:
    import argparse

    import uvicorn

    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--index", default=None, help="saved index path (default: $FM_INDEX_PATH)")
    ap.add_argument("--window-us", type=float, default=200.0, help="batching window")
    args = ap.parse_args()
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(name)s - %(levelname)s - %(message)s")
    uvicorn.run(create_app(index_path=args.index, window_s=args.window_us * 1e-6), host=args.host, port=args.port,
                log_level="error")


if __name__ == "__main__":
    main()
