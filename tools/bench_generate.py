"""The processors' cost inside the hooks the reference actually uses, at C3
(n = 4.5e9 synthetic corpus, B = 256 rows):

* Hugging Face ``generate`` with beam search and ``LogitsProcessorList``
  (/root/reference/index_for_transformers_causal.py:44-62): random-weight
  models of the reference's shapes -- Llama-3.2-1B (vocab 128256) with the
  Causal processor, Qwen3-0.6B (vocab 151936) with the Qwen processor -- 128
  prompts x 2 beams, N new tokens; ms per decode step without a processor,
  with the device path (status event wait, the default), with the device path
  waiting for the whole call (_DeviceStep WAIT_STREAM, round 2's behaviour) and
  with the host path of the same class.  A wrapper times every processor call
  (host wall clock, the call returning).
* vLLM V0's per-sequence hook (/root/reference/index_for_vllm.py:31-32,
  lm_eval_vllm_connection.py:34-35): 256 clones of the Vllm processor, each
  called per step with its whole output tuple and its logits row; the step's
  sampling is one batched argmax (as vLLM samples after the processors); ms
  per step with the tuple-suffix upload (default) vs the whole tuple through
  torch.tensor (round 2).

usage: python tools/bench_generate.py [--tokens 4.5e9] [--new 24] > out.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fm-index-constrained-decoding_amd"))
sys.path.insert(0, REPO)

SHIFT = 10


def log(*a):
    print("[gen]", *a, file=sys.stderr, flush=True)


class Timed:
    """LogitsProcessor wrapper: wall time of every call (the processor returns
    after its own status wait; the caller's next op is stream-ordered)."""

    def __init__(self, proc):
        self.proc = proc
        self.times = []

    def __call__(self, input_ids, scores):
        a = time.perf_counter()
        out = self.proc(input_ids, scores)
        self.times.append(time.perf_counter() - a)
        return out


def build_index(n_tokens, V, dev):
    from fmidx.fm_index import FMIndex
    from fmidx.synth import markov_corpus_gpu

    text, beg = markov_corpus_gpu(n_tokens, V, 20250905, dev)
    fm = FMIndex(device=dev.index)
    fm.initialize_from_text_device(text)
    n = text.numel()
    raw = fm.distinct_count(0, n - 1)
    fm.occurring_distinct = [s - SHIFT for s in raw[0::2] if s > 0]
    return fm, text


def corpus_prompts(text, rows, plen, rng):
    """rows corpus n-grams of F (index.py:47-53: F = reverse(T')) as sentence starts."""
    n = text.numel()
    q = rng.integers(0, n - plen - 2, size=rows)
    idx = torch.tensor((n - 2) - (q[:, None] + np.arange(plen)[None, :]), device=text.device)
    return (text[idx].to(torch.int64) - SHIFT).cpu()


def hf_leg(kind, fm, text, B, beams, new, dev, rng, reps=3):
    from transformers import LlamaConfig, LlamaForCausalLM, LogitsProcessorList, Qwen3Config, Qwen3ForCausalLM

    import fmidx.processors as P

    torch.manual_seed(0)
    if kind == "llama":
        V = 128256
        cfg = LlamaConfig(vocab_size=V, hidden_size=2048, intermediate_size=8192, num_hidden_layers=16,
                          num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=4096,
                          tie_word_embeddings=True, bos_token_id=128000, eos_token_id=128001, pad_token_id=128004)
        with torch.device(dev):
            model = LlamaForCausalLM(cfg).to(torch.bfloat16).eval()
        head = [128000, 882, 2000, 78191, 128007, 271]          # ... the llama-3 end marker [78191, 128007, 271]
        mk = lambda: P.CausalIndexBasedLogitsProcessor(index=fm, num_beams=beams, model_name="llama-3",  # noqa: E731
                                                       pad_token_id=cfg.pad_token_id, eos_token_id=cfg.eos_token_id,
                                                       always_allow_eos=True, length_reward_factor=1.0)
    else:
        V = 151936
        cfg = Qwen3Config(vocab_size=V, hidden_size=1024, intermediate_size=3072, num_hidden_layers=28,
                          num_attention_heads=16, num_key_value_heads=8, head_dim=128, max_position_embeddings=4096,
                          tie_word_embeddings=True, bos_token_id=151643, eos_token_id=151645, pad_token_id=151643)
        with torch.device(dev):
            model = Qwen3ForCausalLM(cfg).to(torch.bfloat16).eval()
        head = [151644, 872, 198, 151645, 198, 151644, 77091, 198, 151667, 271, 151668, 271]
        mk = lambda: P.QwenIndexBasedLogitsProcessor(index=fm, num_beams=beams, min_new_tokens=1,  # noqa: E731
                                                     pad_token_id=cfg.pad_token_id, eos_token_id=cfg.eos_token_id,
                                                     always_allow_eos=True, length_reward_factor=1.0)
    prompts = B // beams
    body = corpus_prompts(text, prompts, 8, rng)
    ids = torch.cat([torch.tensor(head).expand(prompts, -1), body], 1).to(dev)
    att = torch.ones_like(ids)

    def gen(lp, n_new):
        torch.cuda.synchronize()
        a = time.perf_counter()
        with torch.no_grad():
            out = model.generate(ids, attention_mask=att, max_new_tokens=n_new, min_new_tokens=n_new,
                                 num_beams=beams, do_sample=False, logits_processor=lp,
                                 pad_token_id=cfg.pad_token_id, eos_token_id=cfg.eos_token_id,
                                 temperature=None, top_p=None, top_k=None)
        torch.cuda.synchronize()
        return (time.perf_counter() - a), out

    gen(LogitsProcessorList([]), 4)                                    # warm-up (kernels, allocator)
    res = {"model": f"{kind} random weights ({sum(p.numel() for p in model.parameters()) / 1e9:.2f} B params, bf16)",
           "vocab": V, "rows": B, "prompts": prompts, "beams": beams, "new_tokens": new, "reps": reps}
    procs = {}
    for mode in ("event", "stream", "deferred", "host"):
        proc = mk()
        if mode == "host":
            proc._dev = None
        elif mode == "stream":
            proc._dev._wait_stream = True
        elif mode == "deferred":          # no wait for the status (checked at the next call)
            proc._dev._deferred = True
        procs[mode] = Timed(proc)
        gen(LogitsProcessorList([procs[mode]]), 2)                     # first calls: fresh searches, buffers
    # the modes interleaved, `reps` rounds (clock and allocator drift land on every mode alike)
    times = {m: [] for m in ("none", "event", "stream", "deferred", "host")}
    calls = {m: [] for m in ("event", "stream", "deferred", "host")}
    for _ in range(reps):
        for mode in ("none", "event", "stream", "deferred", "host"):
            n_new = new
            if mode == "none":
                t, _ = gen(LogitsProcessorList([]), n_new)
            else:
                w = procs[mode]
                w.times.clear()
                t, _ = gen(LogitsProcessorList([w]), n_new)
                calls[mode].append(float(np.median(w.times)))
                if mode != "host":
                    w.proc._dev.check_pending()
                    assert w.proc._dev.prev_ids is not None, "device path fell back"
            times[mode].append(t / n_new)
    res["no_processor_ms_per_step"] = float(np.median(times["none"])) * 1e3
    for mode in ("event", "stream", "deferred", "host"):
        res[f"{mode}_ms_per_step"] = float(np.median(times[mode])) * 1e3
        res[f"{mode}_ms_per_step_all"] = [x * 1e3 for x in times[mode]]
        res[f"{mode}_processor_ms_per_call"] = float(np.median(calls[mode])) * 1e3
        log(f"{kind} {mode}: {res[f'{mode}_ms_per_step']:.2f} ms/step (no processor "
            f"{res['no_processor_ms_per_step']:.2f}), processor {res[f'{mode}_processor_ms_per_call']:.3f} ms/call")
    res["event_overhead_ms_per_step"] = res["event_ms_per_step"] - res["no_processor_ms_per_step"]
    res["deferred_overhead_ms_per_step"] = res["deferred_ms_per_step"] - res["no_processor_ms_per_step"]
    res["host_overhead_ms_per_step"] = res["host_ms_per_step"] - res["no_processor_ms_per_step"]
    del model
    torch.cuda.empty_cache()
    return res


def vllm_leg(fm, text, seqs, steps, dev, rng):
    import fmidx.processors as P

    V = 151936
    base = P.VllmIndexBasedLogitsProcessor(index=fm, num_beams=1, pad_token_id=151643, eos_token_id=151645,
                                           always_allow_eos=True)
    res = {"sequences": seqs, "steps": steps, "vocab": V}
    per = {}
    for mode in ("suffix", "tensor"):
        clones = [base.clone() for _ in range(seqs)]
        if mode == "tensor":      # round 2: the whole tuple through torch.tensor + a pageable copy every call
            for c in clones:
                c._device_ids = lambda toks, c=c: torch.tensor([list(toks)], dtype=torch.long)
        per[mode] = (clones, [[] for _ in range(seqs)], [])
    logits = torch.randn((seqs, V), device=dev).to(torch.bfloat16)
    for s in range(steps):
        for mode in ("suffix", "tensor"):            # interleaved step by step
            clones, outs, per_step = per[mode]
            torch.cuda.synchronize()
            a = time.perf_counter()
            rows = [clones[i](tuple(outs[i]), logits[i]) for i in range(seqs)]
            nxt = torch.cat(rows).float().argmax(1).tolist()        # vLLM samples once, after every processor
            per_step.append(time.perf_counter() - a)
            for i, t in enumerate(nxt):
                outs[i].append(int(t))
    for mode in ("suffix", "tensor"):
        res[f"{mode}_ms_per_step"] = float(np.median(per[mode][2][2:])) * 1e3
        res[f"{mode}_ms_per_call"] = res[f"{mode}_ms_per_step"] / seqs
        log(f"vllm {mode}: {res[f'{mode}_ms_per_step']:.2f} ms per step of {seqs} calls")
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--beams", type=int, default=2)
    ap.add_argument("--new", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--models", default="llama,qwen")
    ap.add_argument("--vllm-seqs", type=int, default=256)
    ap.add_argument("--vllm-steps", type=int, default=12)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.time()
    fm, text = build_index(int(args.tokens), 128256, dev)
    log(f"index n={fm.size()} in {time.time() - t0:.1f}s")
    rng = np.random.default_rng(5)
    result = {"n": fm.size(), "hf": {}}
    for kind in args.models.split(","):
        result["hf"][kind] = hf_leg(kind, fm, text, args.batch, args.beams, args.new, dev, rng, args.reps)
    result["vllm"] = vllm_leg(fm, text, args.vllm_seqs, args.vllm_steps, dev, rng)
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
