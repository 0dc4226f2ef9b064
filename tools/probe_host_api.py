"""Per-call latency of the synchronous host-API batch calls (get_range_batch,
distinct_count_multi, backward_search_multi) on a small index: the cost the
processors pay once per decode step.  FMIDX_LIB selects the library."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
from fmidx.index import FMIndex  # noqa: E402

rng = np.random.default_rng(1)
docs = [rng.integers(0, 5000, size=int(rng.integers(50, 500))).tolist() for _ in range(2000)]
ix = FMIndex(device=0)  # FMIDX_LIB: absolute path of the library to load
ix.initialize(docs, in_memory=True)
F = [t for d in reversed(docs) for t in d]
pats = [F[s: s + 8] for s in rng.integers(0, len(F) - 9, size=256)]


def per_call(fn, reps=200):
    for _ in range(10):
        fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps * 1e6


lo, hi = ix.get_range_batch(pats, 10)
raw = ix      # index.FMIndex is the SWIG-surface class plus index.py
out = {"lib": os.path.basename(os.environ.get("FMIDX_LIB", "libfmidx.so")),
       "get_range_batch_256x8_us": per_call(lambda: ix.get_range_batch(pats, 10))}
if raw is not None:
    out["distinct_count_multi_256_us"] = per_call(lambda: raw.distinct_count_multi(lo.tolist(), hi.tolist()), 50)
    out["backward_search_multi_8_us"] = per_call(lambda: raw.backward_search_multi([t + 10 for t in pats[0]]))
    out["backward_search_step_us"] = per_call(lambda: raw.backward_search_step(pats[0][0] + 10, 0, ix.size() - 1))
print(out, flush=True)
