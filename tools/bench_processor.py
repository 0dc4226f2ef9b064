"""Per-call latency of one logits-processor step (the reference's hook,
document_constrained_generation_causal_qwen.py:101-214) on the MI355X engine:
QwenIndexBasedLogitsProcessor.__call__ on B rows x V vocab scores, rows
decoding true continuations of the indexed corpus (p = 0.9, else a random id).
The whole per-call cost a generate() loop sees (input_ids already on the
device): the per-row bookkeeping, the pattern ranges, the packed mask, the
fused epilogue -- on the device path (fm_processor_step) and, for comparison,
the host path of the same class.
Usage: python tools/bench_processor.py [--tokens N] [--batch B] [--vocab V] [--dtype bf16|f32]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import fmidx.processors as P  # noqa: E402
from fmidx.fm_index import suffix_sort_device  # noqa: E402
from fmidx.index import FMIndex  # noqa: E402
from fmidx.synth import markov_corpus_gpu  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tokens", type=float, default=4.5e9)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--vocab", type=int, default=128256)
ap.add_argument("--dtype", default="bf16")
ap.add_argument("--steps", type=int, default=24)
ap.add_argument("--host-steps", type=int, default=6)
ap.add_argument("--variant", default="qwen", choices=["qwen", "seq"],
                help="qwen: QwenIndexBasedLogitsProcessor (soft); seq: SeqIndexBasedLogitsProcessor (hard mask)")
args = ap.parse_args()
B, V = args.batch, args.vocab
DT = {"f32": torch.float32, "bf16": torch.bfloat16}[args.dtype]
dev = torch.device("cuda", 0)
SHIFT = 10

t0 = time.perf_counter()
text, beg = markov_corpus_gpu(int(args.tokens), V, 20250905, dev)
bwt, _ = suffix_sort_device(text)
ix = FMIndex(device=0)
ix.initialize_from_bwt_device(bwt)
ix.beginnings = beg.cpu().tolist()
ix.occurring_distinct, ix.occurring_counts = ix.get_distinct_count(0, len(ix))
build_s = time.perf_counter() - t0
n = text.numel()

head = [151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]   # end marker + system/think tokens
g = torch.Generator(device=dev)
g.manual_seed(3)
q = torch.randint(0, n - 2000, (B,), generator=g, device=dev)
# row b decodes F = reverse(T') from position q[b]: F[q + k] = T'[n - 2 - q - k]
steps = args.steps + args.host_steps + 4
k = torch.arange(steps + 4, device=dev)
true = (text[(n - 2) - (q[:, None] + k[None, :])].to(torch.int64) - SHIFT).cpu().numpy()
del text, bwt
torch.cuda.empty_cache()
rng = np.random.default_rng(7)
sents = [[int(true[b, 0])] for b in range(B)]
ids_seq = []
for s in range(steps):
    for b in range(B):
        sents[b].append(int(true[b, len(sents[b])]) if rng.random() < 0.9 else int(rng.integers(3, V - 20)))
    pre = head if args.variant == "qwen" else [1]     # seq2seq rows start with the decoder start token
    ids_seq.append(torch.tensor([pre + x for x in sents], dtype=torch.int64, device=dev))
scores = torch.randn(B, V, device=dev).to(DT)


def run(proc, seq, warm):
    times = []
    for i, ids in enumerate(seq):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = proc(ids, scores)
        torch.cuda.synchronize()
        if i >= warm:
            times.append(time.perf_counter() - t)
    return np.array(times) * 1e3, out


kw = dict(index=ix, num_beams=1, pad_token_id=0, eos_token_id=2)
Proc = P.QwenIndexBasedLogitsProcessor if args.variant == "qwen" else P.SeqIndexBasedLogitsProcessor
proc = Proc(**kw)
assert proc._dev is not None
td, out_d = run(proc, ids_seq[: 4 + args.steps], 4)
host = Proc(**kw)
host._dev = None
th, out_h = run(host, ids_seq[: 4 + args.host_steps], 2)
same = bool(torch.equal(out_d.view(torch.int16 if DT != torch.float32 else torch.int32),
                        Proc(**kw)(ids_seq[3 + args.steps], scores)
                        .view(torch.int16 if DT != torch.float32 else torch.int32)))
res = {"variant": args.variant, "B": B, "V": V, "dtype": args.dtype, "corpus_tokens": n, "index_build_s": round(build_s, 1),
       "device_path": {"steps": len(td), "ms_per_call_mean": round(float(td.mean()), 4),
                       "ms_per_call_median": round(float(np.median(td)), 4), "ms_per_call_min": round(float(td.min()), 4),
                       "ms_per_call_max": round(float(td.max()), 4), "rows_per_s": round(B / (td.mean() / 1e3))},
       "host_path": {"steps": len(th), "ms_per_call_mean": round(float(th.mean()), 3),
                     "ms_per_call_median": round(float(np.median(th)), 3)},
       "incremental_equals_fresh": same, "pattern_len_at_end": len(sents[0])}
print(json.dumps(res), flush=True)
