#!/usr/bin/env python
"""bench.py -- allowed-token masks/s of the FM-index decode step on MI355X.

One step = one decode step of the hot path for B rows: the LF (backward-search)
update of every row's (low, high) range by its new token, then the
allowed-next-token mask bool[B, V] of the new ranges (SURVEY §8a A2-A8,
incremental mode of §5 "long-context").  Inputs (index, decode trace,
states) are resident in HBM before timing.

Workload (BASELINE configs[2]: n = 4.5e9 "enwiki" scale, B = 256): seeded order-1 Markov corpus with Zipf(1.1) rows over
V = 128256 (+SHIFT 10, 17 wavelet levels), lognormal docs (mean ~500),
encoded exactly as index.py:47-53; suffix array built on the GPU.  Decode
trace: B rows start from U{1..32}-token true corpus patterns; each step a row
appends a true continuation (a random occurrence's next token, p = 0.9) or a
uniform random id; a row whose range is empty restarts as a fresh sequence
(empty pattern = full range); row 0 is an empty-pattern row, row 1 an
eos-terminated (empty-range) row.

Multi-GPU (--gpus N under torch.distributed.run): replicas -- every rank holds
the full index and decodes its own B rows (weak scaling, no data-path
collective); value = N*B*K / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "fm-index-constrained-decoding_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from fmidx.fm_index import FMIndex, suffix_sort_device, wt_int_levels_device  # noqa: E402
from fmidx.synth import markov_corpus_gpu  # noqa: E402

SHIFT = 10
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 measured stream)
HBM_STREAM_GBS = 6290.0   # measured stream rate (MI355X_MICROARCH.md)
METRIC = "allowed-token masks/sec @ B=256, 128k vocab"


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
def build_index(n_tokens: int, vocab: int, seed: int, dev):
    t0 = time.time()
    text, beg = markov_corpus_gpu(n_tokens, vocab, seed, dev)
    torch.cuda.synchronize()
    t1 = time.time()
    log(f"corpus n={text.numel()} docs={beg.numel() - 1} in {t1 - t0:.1f}s; GPU suffix sorting ...")
    bwt, _ = suffix_sort_device(text)      # csrc/sa.hip: prefix doubling, 64-bit positions
    torch.cuda.synchronize()
    t2 = time.time()
    log(f"suffix sorting {t2 - t1:.1f}s; building the index ...")
    fm = FMIndex(device=dev.index)
    fm.initialize_from_bwt_device(bwt)
    torch.cuda.synchronize()
    t3 = time.time()
    log(f"corpus {t1 - t0:.1f}s  suffix array {t2 - t1:.1f}s  index {t3 - t2:.1f}s  n={bwt.numel()}")
    return fm, text, bwt, {"corpus_s": t1 - t0, "sa_s": t2 - t1, "index_s": t3 - t2}


def make_trace(fm, text, bwt, B: int, V: int, S: int, seed: int, dev):
    """Decode trace (untimed): tokens[S, B] (-1 = restart as a fresh sequence)
    and the states after every step (for byte accounting and the CPU leg)."""
    g = torch.Generator(device=dev)
    g.manual_seed(seed + 1)
    n = bwt.numel()
    # initial patterns: true corpus n-grams of F = reverse(T') (the text patterns match)
    lens = torch.randint(1, 33, (B,), generator=g, device=dev)
    q = torch.randint(0, n - 40, (B,), generator=g, device=dev)
    offs = torch.zeros(B + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    tot = int(offs[-1].item())
    row_of = torch.repeat_interleave(torch.arange(B, device=dev), lens)
    k = torch.arange(tot, device=dev) - offs[:-1][row_of]
    fpos = q[row_of] + k                              # F position
    toks = text[(n - 2) - fpos].to(torch.int64) - SHIFT
    lo = torch.zeros(B, dtype=torch.int64, device=dev)
    hi = torch.zeros(B, dtype=torch.int64, device=dev)
    fm.backward_search_batch(toks, offs, SHIFT, lo, hi)
    lo[0], hi[0] = 0, n          # empty-pattern row
    lo[1], hi[1] = 0, 0          # eos-terminated row
    init = (lo.clone(), hi.clone())
    tokens = torch.empty((S, B), dtype=torch.int64, device=dev)
    lo_hist = torch.empty((S, B), dtype=torch.int64, device=dev)
    hi_hist = torch.empty((S, B), dtype=torch.int64, device=dev)
    dummy = torch.empty((1, 1), dtype=torch.uint8, device=dev)
    for s in range(S):
        live = lo < hi
        width = (hi - lo).clamp(min=1)
        u = torch.rand(B, generator=g, device=dev, dtype=torch.float64)
        j = (lo + (u * width.to(torch.float64)).to(torch.int64).clamp(max=n - 1)).clamp(max=n - 1)
        true_tok = bwt[j].to(torch.int64) - SHIFT
        rnd = torch.randint(0, V, (B,), generator=g, device=dev)
        coin = torch.rand(B, generator=g, device=dev) < 0.9
        tok = torch.where(coin & (true_tok >= 0), true_tok, rnd)
        tok = torch.where(live, tok, torch.full_like(tok, -1))
        tok[0] = -1
        tok[1] = V + 1000             # unknown id: the eos row stays empty
        tokens[s] = tok
        fm.decode_step(tok, lo, hi, dummy, 0, SHIFT, reset_below=0)
        lo_hist[s] = lo
        hi_hist[s] = hi
    torch.cuda.synchronize()
    return tokens, init, lo_hist, hi_hist


def plan_bytes(lo: np.ndarray, hi: np.ndarray, n: int, b0_log2: int, bm_levels: int, bm_bytes_each: int,
               follow=None, cached=None):
    """Bytes the mask algorithm must read per row: one cached range bitmap,
    or streamed BWT symbols (4 B) + whole aligned bitmaps (mirrors the plan
    of k_decode in decode.hip)."""
    B0 = 1 << b0_log2
    out = np.zeros(lo.size, dtype=np.int64)
    for i, (l, h) in enumerate(zip(lo.tolist(), hi.tolist())):
        h = min(h, n)
        if l >= h:
            continue
        if (cached is not None and cached[i]) or (l == 0 and h == n) or (follow is not None and follow[i]):
            out[i] = bm_bytes_each            # one precomputed bitmap (full range / follow set)
            continue
        if bm_levels == 0 or h - l <= B0:
            out[i] = 4 * (h - l)
            continue
        x = (l + B0 - 1) >> b0_log2
        y = h >> b0_log2
        if x >= y:
            out[i] = 4 * (h - l)
            continue
        nb = 0
        while x < y:
            j = 0
            while j + 1 < bm_levels:
                span = 1 << (2 * (j + 1))
                if (x & (span - 1)) or x + span > y:
                    break
                j += 1
            nb += 1
            x += 1 << (2 * j)
        out[i] = 4 * (((((l + B0 - 1) >> b0_log2) << b0_log2) - l) + (h - ((h >> b0_log2) << b0_log2))) \
            + nb * bm_bytes_each
    return out


# ---------------------------------------------------------------------------
def cpu_baseline(fm, bwt, tokens, lo_hist, hi_hist, V, warmup, seconds, dev):
    """The sdsl-faithful C++ restatement (oracle/cpu_ref.cpp) on the host
    cores, replaying the same trace from step `warmup` until ~`seconds`; its
    final ranges AND its final step's masks are compared with the GPU's (a
    full-scale bit-exact check against an independent implementation)."""
    from oracle.cpu_ref import CpuRef

    n = bwt.numel()
    L = max(1, int(bwt.max().item()).bit_length())
    # sdsl wt_int level bit vectors built on the GPU (csrc/sa.hip), copied to the host
    words = wt_int_levels_device(bwt, L).cpu().numpy().view(np.uint64)
    cnt = torch.bincount(bwt.to(torch.int64), minlength=(1 << L) + 1)
    C = torch.zeros((1 << L) + 1, dtype=torch.int64, device=dev)
    torch.cumsum(cnt[: 1 << L], 0, out=C[1:])
    sigma = int((cnt > 0).sum().item())
    C = C.cpu().numpy().view(np.uint64)
    del cnt
    t0 = time.time()
    ref = CpuRef(words, n, L, C, sigma)
    log(f"cpu_ref build {time.time() - t0:.1f}s")
    threads = int(os.environ.get("FMIDX_CPU_THREADS", min(16, os.cpu_count() or 1)))
    B = tokens.shape[1]
    tok_np = tokens.cpu().numpy()
    lo = lo_hist[warmup - 1].cpu().numpy().astype(np.uint64) if warmup > 0 else None
    hi = hi_hist[warmup - 1].cpu().numpy().astype(np.uint64) if warmup > 0 else None
    mask = np.zeros((B, V), dtype=np.uint8)
    rows = 0
    steps = 0
    t0 = time.time()
    s = warmup
    while s < tok_np.shape[0]:
        ref.decode_step(np.ascontiguousarray(tok_np[s]), SHIFT, 0, lo, hi, mask, threads)
        rows += B
        steps += 1
        s += 1
        if time.time() - t0 >= seconds:
            break
    el = time.time() - t0
    ok = bool(np.array_equal(lo, lo_hist[s - 1].cpu().numpy().astype(np.uint64)) and
              np.array_equal(hi, hi_hist[s - 1].cpu().numpy().astype(np.uint64)))
    # the GPU's mask of the same step (s - 1), from the same incoming state
    gmask = torch.empty((B, V), dtype=torch.uint8, device=dev)
    glo = torch.empty(B, dtype=torch.int64, device=dev)
    ghi = torch.empty(B, dtype=torch.int64, device=dev)
    fm.decode_step(tokens[s - 1], lo_hist[s - 2], hi_hist[s - 2], gmask, V, SHIFT, reset_below=0,
                   lo_out=glo, hi_out=ghi)
    mok = bool(np.array_equal(mask, gmask.cpu().numpy()))
    return {"value": rows / el, "unit": "masks/s", "cores": threads, "kind": "port",
            "sample": f"{steps} decode steps x {B} rows of the same trace (steps {warmup}..{s - 1}), "
                      f"same n={n} index, sdsl-faithful wt_int + rank_support_v restatement, "
                      f"{threads} threads, {el:.1f}s; final ranges match GPU: {ok}; "
                      f"final step's {B}x{V} masks match GPU: {mok}",
            "ranges_match_gpu": ok, "masks_match_gpu": mok}


# ---------------------------------------------------------------------------
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--tokens", type=float, default=float(os.environ.get("FMIDX_BENCH_TOKENS", 4.5e9)))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--seed", type=int, default=20250905)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-steps", type=int, default=600)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--packed", action="store_true",
                    help="bit-packed masks (uint32[B, ceil(V/32)]) instead of uint8[B, V] (not the headline)")
    ap.add_argument("--dump-trace", default="", help="write the timed trace states to this .npz")
    ap.add_argument("--eager-replay", action="store_true",
                    help="after the timed region, launch the K timed steps once more eagerly (no graph) "
                         "so PMC counters can be collected per dispatch (tools/pmc_traffic.sh)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU: bind the device BEFORE the RCCL communicator exists
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
    n_tokens = int(args.tokens)
    B, V, K, W = args.batch, args.vocab, args.steps, max(1, args.warmup)

    fm, text, bwt, build_t = build_index(n_tokens, V, args.seed, dev)
    n = bwt.numel()
    st = fm.stats()
    S = W + K
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu and args.cpu_seconds > 0
    # the CPU leg replays the same trace past the GPU's steps (bounded by time)
    S_trace = S + (args.cpu_steps if cpu_leg else 0)
    tokens, init, lo_hist, hi_hist = make_trace(fm, text, bwt, B, V, S_trace, args.seed + rank, dev)
    del text
    PK = bool(args.packed)
    mask = (torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev) if PK
            else torch.empty((B, V), dtype=torch.uint8, device=dev))
    lo = init[0].clone()
    hi = init[1].clone()
    dummy = torch.empty((1, 1), dtype=torch.uint8, device=dev)

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    for s in range(W):
        fm.decode_step(tokens[s], lo, hi, mask, V, SHIFT, reset_below=0, packed=PK)
    torch.cuda.synchronize()
    state_lo, state_hi = lo.clone(), hi.clone()

    # Capture the K timed steps into one HIP graph (the C-ABI launches go onto
    # torch's capture stream): one fused k_decode launch per step (LF step +
    # allowed mask), ping-ponging the (lo, hi) state buffers.  Per-kernel
    # graphs for the roofline: K standalone LF launches and K mask-only
    # launches on the recorded states.  Replays are timed with HIP events.
    bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]
    lo_scr = torch.empty_like(lo)
    hi_scr = torch.empty_like(hi)
    g_step = torch.cuda.CUDAGraph()
    g_lf = torch.cuda.CUDAGraph()
    g_mask = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_step):
        for i in range(K):
            src, dst = bufs[i % 2], bufs[(i + 1) % 2]
            fm.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0,
                           lo_out=dst[0], hi_out=dst[1], packed=PK)
    with torch.cuda.graph(g_lf):
        for i in range(K):
            fm.lf_step_batch(tokens[W + i], lo_hist[W + i - 1], hi_hist[W + i - 1], SHIFT,
                             lo_out=lo_scr, hi_out=hi_scr, reset_below=0)
    with torch.cuda.graph(g_mask):
        for i in range(K):
            fm.allowed_mask(lo_hist[W + i], hi_hist[W + i], V, SHIFT, out=mask, packed=PK)

    def timed(graph, reps=1, reset=False):
        ts = []
        for _ in range(reps):
            if reset:
                lo.copy_(state_lo)
                hi.copy_(state_hi)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            graph.replay()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return ts

    # standalone kernels first, so that the fused step's own replays (which
    # also warm its code, caches and TLB) come right before the timed region
    lf_ms = [t / K for t in timed(g_lf, 5)]
    mask_ms = [t / K for t in timed(g_mask, 5)]
    step_reps = timed(g_step, 3, reset=True)
    lo.copy_(state_lo)
    hi.copy_(state_hi)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    wall0 = time.time()
    t_start = torch.cuda.Event(enable_timing=True)
    t_end = torch.cuda.Event(enable_timing=True)
    t_start.record()
    g_step.replay()
    t_end.record()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    wall = time.time() - wall0
    elapsed_ms = t_start.elapsed_time(t_end)
    fin = bufs[K % 2]
    ok = bool(torch.equal(fin[0], lo_hist[S - 1]) and torch.equal(fin[1], hi_hist[S - 1]))
    step_ms = elapsed_ms / K
    if world > 1:
        import torch.distributed as dist

        t = torch.tensor([step_ms], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        step_ms = float(t.item())
    value = world * B * K / (step_ms * K / 1e3)

    if args.eager_replay:
        lo.copy_(state_lo)
        hi.copy_(state_hi)
        for i in range(K):
            src, dst = bufs[i % 2], bufs[(i + 1) % 2]
            fm.decode_step(tokens[W + i], src[0], src[1], mask, V, SHIFT, reset_below=0,
                           lo_out=dst[0], hi_out=dst[1], packed=PK)
        torch.cuda.synchronize()
    if args.dump_trace and rank == 0:
        np.savez_compressed(args.dump_trace, tokens=tokens[:S].cpu().numpy(), lo=lo_hist[:S].cpu().numpy(),
                            hi=hi_hist[:S].cpu().numpy(), n=n, warmup=W)
    # ---- roofline accounting for the dominant (mask) kernel
    lo_np = lo_hist[W:S].cpu().numpy()
    hi_np = hi_hist[W:S].cpu().numpy()
    max_sym = int(bwt.max().item())
    words = ((max_sym + 1 + 127) // 128) * 4
    b0 = st["bitmap_block"]
    b0_log2 = b0.bit_length() - 1 if b0 else 0
    nb0 = n >> b0_log2 if b0 else 0
    bm_levels = 0
    c = nb0
    while c > 0:
        bm_levels += 1
        c >>= 2
    prev_lo = np.concatenate([lo_hist[W - 1:W].cpu().numpy(), lo_np[:-1]])
    prev_hi = np.concatenate([hi_hist[W - 1:W].cpu().numpy(), hi_np[:-1]])
    tok_np = tokens[W:S].cpu().numpy()
    follow = (prev_lo == 0) & (prev_hi >= n) & (tok_np >= 0) & (st.get("follow_bytes", 0) > 0)
    cached = fm.cache_contains(lo_hist[W:S].reshape(-1).contiguous(),
                               hi_hist[W:S].reshape(-1).contiguous()).view(K, B).cpu().numpy()
    read_bytes = np.stack([plan_bytes(lo_np[i], hi_np[i], n, b0_log2, bm_levels, words * 4, follow[i], cached[i])
                           for i in range(K)])
    mask_bytes_per_launch = float((read_bytes.sum(1) + (B * ((V + 31) // 32) * 4 if PK else B * V)).mean())
    mask_us = float(np.median(mask_ms)) * 1e3
    NL = st["levels"]
    # LF: per digit level and endpoint one 128-B rank block + one 8-B
    # superblock count, for every row that was live (restarts cost nothing)
    live = (prev_lo < prev_hi) & (tok_np >= 0)
    lf_bytes = (128 + 8) * 2 * NL * live.sum(1)
    lf_us = float(np.median(lf_ms)) * 1e3
    rank_gbs = float(lf_bytes.mean()) / (lf_us * 1e-6) / 1e9
    # dominant kernel = the fused k_decode (one launch per step)
    decode_bytes = mask_bytes_per_launch + float(lf_bytes.mean())
    decode_us = step_ms * 1e3
    achieved = decode_bytes / (decode_us * 1e-6) / 1e9
    widths = (hi_np - lo_np)
    log(f"step {step_ms * 1e3:.1f}us [reps {', '.join(f'{t / K * 1e3:.1f}' for t in step_reps)}] "
        f"(standalone lf {lf_us:.1f}us, mask {mask_us:.1f}us, wall/step {wall / K * 1e6:.1f}us, graph) "
        f"bytes/step {decode_bytes / 1e6:.2f}MB -> {achieved:.0f} GB/s; "
        f"live rows {(widths > 0).mean():.2f}, median width {np.median(widths[widths > 0]) if (widths > 0).any() else 0}, "
        f"cached rows {cached.mean():.3f} (cache: {st['cache_nodes']} ranges >= {st['cache_min']}, "
        f"{st['cache_bytes'] / 2**30:.1f} GiB; transitions {st['trans_entries']} "
        f"(+{st['trans_dropped']} left out), {st['trans_bytes'] / 2**30:.1f} GiB)")

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "masks/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "uint64",
        "data": "synthetic",
        "config": {
            "workload": f"decode step (LF + allowed-token mask) over a synthetic Markov/Zipf corpus "
                        f"of n={n} tokens ({'C3 enwiki' if n > 2e9 else ('C5 PAQ' if n > 1e9 else 'C2 simplewiki')} "
                        f"scale), B={B} rows, V={V}, incremental ranges",
            "corpus_tokens": n,
            "global_batch": world * B,
            "batch_per_gpu": B,
            "vocab": V,
            "wavelet_digit_levels": NL,
            "parallelism": f"replicas{world}",
            "mask": "uint32[B,ceil(V/32)] bit-packed" if PK else "uint8[B,V]",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "k_decode (fused LF step + allowed mask)",
            "alg_bytes_per_launch": decode_bytes,
            "avg_launch_us": decode_us,
            # also against the measured stream rate of MI355X_MICROARCH.md
            "peak_stream_measured": HBM_STREAM_GBS,
            "frac_stream": achieved / HBM_STREAM_GBS,
        },
        "standalone_kernels": {
            "k_lf": {"avg_launch_us": lf_us, "rank_GBps": rank_gbs, "alg_bytes_per_launch": float(lf_bytes.mean())},
            "k_decode_mask_only": {"avg_launch_us": mask_us, "alg_bytes_per_launch": mask_bytes_per_launch,
                                   "GBps": mask_bytes_per_launch / (mask_us * 1e-6) / 1e9},
        },
        "index": {"build": build_t, **st},
        "trace_check": ok,
    }
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                t = json.load(f)
            if t.get("corpus_tokens") == n and t.get("batch") == B:
                result["roofline"]["traffic"] = t.get("k_decode_bytes_per_launch")
        except Exception:
            pass
    if cpu_leg:
        try:
            result["cpu_baseline"] = cpu_baseline(fm, bwt, tokens, lo_hist, hi_hist, V, W, args.cpu_seconds, dev)
        except Exception as e:  # the GPU line must still print
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
