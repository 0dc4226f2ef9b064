"""Per-call latency of one logits-processor step (the reference's hook,
document_constrained_generation_causal_qwen.py:101-214) on the MI355X engine:
QwenIndexBasedLogitsProcessor.__call__ on B rows x V vocab scores, rows
decoding true continuations of indexed documents (p = 0.9, else a random id).
Covers the whole per-step cost a generate() loop sees: the D2H of input_ids,
the per-row Python bookkeeping, the batched range search, the packed mask and
the fused epilogue.  Usage: python tools/bench_processor.py [B] [V] [dtype]"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import fmidx.processors as P  # noqa: E402
from fmidx.index import FMIndex  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
V = int(sys.argv[2]) if len(sys.argv) > 2 else 128256
DT = {"f32": torch.float32, "bf16": torch.bfloat16}[sys.argv[3] if len(sys.argv) > 3 else "bf16"]
STEPS, WARM = 24, 4

rng = np.random.default_rng(7)
zipf = np.minimum(rng.zipf(1.1, size=3_000_000), V - 20) + 3
docs, o = [], 0
while o < len(zipf) - 1000:
    n = int(rng.integers(100, 600))
    docs.append(zipf[o:o + n].tolist())
    o += n
t0 = time.perf_counter()
ix = FMIndex()
ix.initialize(docs, in_memory=True)
build_s = time.perf_counter() - t0
F = [t for d in reversed(docs) for t in d]

head = [151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]   # end marker + system/think tokens
starts = rng.integers(0, len(F) - 200, size=B)
sents = [[F[int(s)]] for s in starts]
proc = P.QwenIndexBasedLogitsProcessor(index=ix, num_beams=1, pad_token_id=0, eos_token_id=2)
dev = torch.device("cuda", 0)
scores = torch.randn(B, V, device=dev).to(DT)
times = []
for step in range(WARM + STEPS):
    for b in range(B):
        if rng.random() < 0.9:
            pos = int(starts[b]) + len(sents[b])
            sents[b].append(F[pos] if pos < len(F) else 5)
        else:
            sents[b].append(int(rng.integers(3, V - 20)))
    ids = torch.tensor([head + s for s in sents], dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = proc(ids, scores)
    torch.cuda.synchronize()
    times.append(time.perf_counter() - t)
t = np.array(times[WARM:]) * 1e3
print({"B": B, "V": V, "dtype": str(DT).split(".")[1], "corpus_tokens": len(F), "index_build_s": round(build_s, 2),
       "steps": STEPS, "ms_per_call_mean": round(float(t.mean()), 3), "ms_per_call_median": round(float(np.median(t)), 3), "ms_per_call_min": round(float(t.min()), 3),
       "ms_per_call_max": round(float(t.max()), 3), "rows_per_s": round(B / (t.mean() / 1e3)),
       "pattern_len_at_end": len(sents[0])}, flush=True)
