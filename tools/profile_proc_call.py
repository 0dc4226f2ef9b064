#!/usr/bin/env python
"""Host cost of one processor call (the per-call Python + ctypes work the
reference hooks pay on top of the device work): vLLM V0's per-sequence hook
(one Vllm processor clone per sequence, one call per step with the whole
output tuple) and a Causal / Qwen call at B = 256, each timed over many calls
on a small index (the device work is a few us; the host work is what is
measured), with a cProfile summary of the vLLM calls.

    python tools/profile_proc_call.py [--calls 4000] [--profile]
"""
from __future__ import annotations

import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fm-index-constrained-decoding_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4000)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    import fmidx.processors as P
    from fmidx.index import FMIndex

    rng = np.random.default_rng(0)
    docs = [rng.integers(0, 5000, size=int(rng.integers(50, 400))).tolist() for _ in range(3000)]
    ix = FMIndex(device=0)
    ix.initialize(docs, in_memory=True)
    F = [t for d in reversed(docs) for t in d]
    dev = torch.device("cuda", 0)
    V = 151936
    res = {}
    # vLLM V0: 64 clones, each called with its growing output tuple
    base = P.VllmIndexBasedLogitsProcessor(index=ix, num_beams=1, pad_token_id=151643, eos_token_id=151645,
                                           always_allow_eos=True)
    seqs = 64
    clones = [base.clone() for _ in range(seqs)]
    starts = rng.integers(0, len(F) - 500, size=seqs)
    logits = torch.randn((seqs, V), device=dev).to(torch.bfloat16)
    outs = [[] for _ in range(seqs)]
    steps = max(2, args.calls // seqs)

    def run_steps(n):
        for _ in range(n):
            for i in range(seqs):
                clones[i](tuple(outs[i]), logits[i])
            for i in range(seqs):
                outs[i].append(F[int(starts[i]) + len(outs[i])])

    run_steps(2)
    torch.cuda.synchronize()
    a = time.perf_counter()
    run_steps(steps)
    torch.cuda.synchronize()
    res["vllm_us_per_call"] = (time.perf_counter() - a) / (steps * seqs) * 1e6
    if args.profile:
        pr = cProfile.Profile()
        pr.enable()
        run_steps(8)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
        print(s.getvalue(), file=sys.stderr)
    # soft processors at B = 256 (4 beams): one call per step, the call's host wall and the step's
    for kind in ("causal", "qwen"):
        B, beams = 256, 4
        if kind == "qwen":
            head = [151644, 872, 198, 151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]
            proc = P.QwenIndexBasedLogitsProcessor(index=ix, num_beams=beams, min_new_tokens=1, pad_token_id=151643,
                                                   eos_token_id=151645, always_allow_eos=True, length_reward_factor=1.0)
        else:
            head = [128000, 882, 78191, 128007, 271]
            proc = P.CausalIndexBasedLogitsProcessor(index=ix, num_beams=beams, model_name="llama-3",
                                                     pad_token_id=0, eos_token_id=2, always_allow_eos=True,
                                                     length_reward_factor=1.0)
        st = rng.integers(0, len(F) - 500, size=B)
        sents = [list(F[s:s + 4]) for s in st]
        scores = torch.randn((B, V), device=dev).to(torch.bfloat16)
        walls = []
        for step in range(40):
            ids = torch.tensor([head + s for s in sents], dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            a = time.perf_counter()
            proc(ids, scores)
            walls.append(time.perf_counter() - a)
            for b in range(B):
                sents[b].append(F[int(st[b]) + len(sents[b])])
        res[f"{kind}_call_ms_idle_gpu"] = float(np.median(walls[5:])) * 1e3
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
