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

Multi-GPU (--gpus N): replicas -- every rank holds the full index and decodes
its own B rows (weak scaling, no data-path collective); value = N*B*K /
max-over-ranks time.  Launched either by torch.distributed.run (WORLD_SIZE in
the environment) or plainly as ``python bench.py --gpus N``: then this process
never touches the GPU -- it starts N fresh child processes (one per GPU, RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set), waits for
them and exits with the worst exit code (spawn_ranks).  After the replica
run, N > 1 also runs the doc-range sharded config (C4) over RCCL.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import threading
import time
import traceback

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "fm-index-constrained-decoding_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from fmidx._lib import check, lib  # noqa: E402
from fmidx.fm_index import FMIndex  # noqa: E402
from fmidx.synth import decode_trace, markov_corpus_gpu, paq_corpus_gpu, paq_trace, trace_patterns  # noqa: E402

SHIFT = 10
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 measured stream)
HBM_STREAM_GBS = 6290.0   # measured stream rate (MI355X_MICROARCH.md)
METRIC = "allowed-token masks/sec @ B=256, 128k vocab"


def lib_sha16():
    import hashlib

    with open(os.path.join(PKG, "fmidx", "libfmidx.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus(env: dict | None = None, topology: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs this process could use, counted WITHOUT the HIP runtime (the
    launcher parent must not initialise the GPU: torch.cuda.device_count() asks
    amdsmi first but falls back to a HIP runtime call): the KFD topology nodes
    with a nonzero gpu_id, limited by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES
    / CUDA_VISIBLE_DEVICES when set (an empty list hides every GPU)."""
    import glob

    env = os.environ if env is None else env
    n = 0
    for path in glob.glob(os.path.join(topology, "*", "gpu_id")):
        try:
            with open(path) as f:
                n += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if var in env:
            ids = [x for x in env[var].split(",") if x.strip()]
            n = min(n, len(ids))
    return n


def spawn_ranks(n: int, cmd: list, grace_s: float = 30.0, env: dict | None = None) -> int:
    """One fresh child process per GPU running ``cmd`` with the torchrun-style
    rank environment; returns the worst exit code.  The caller must not have
    touched the GPU (no HIP call, no torch.cuda.is_available()): the children
    are started as new programs, never by exec of this one.  When a child fails,
    the others get ``grace_s`` to finish on their own (a rank stuck in a
    collective with a dead peer would otherwise wait for the RCCL timeout), then
    are terminated by PID.  Returns the first failing rank's code (the cause),
    not the SIGTERM of the peers stopped after it."""
    import signal
    import subprocess

    port = free_port()
    procs = []
    for r in range(n):
        e = dict(os.environ if env is None else env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                  "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                  "FMIDX_BENCH_LAUNCHER": "spawn"})
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")      # RCCL on this host needs dmabuf IPC
        procs.append(subprocess.Popen(cmd, env=e))
    codes = [None] * n
    fail_at, first_bad = None, 0
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
                if codes[i] not in (None, 0) and fail_at is None:
                    fail_at, first_bad = time.time(), codes[i]
                    print(f"[bench] rank {i} exited with {codes[i]}", file=sys.stderr, flush=True)
        if fail_at is not None and time.time() - fail_at > grace_s:
            for i, p in enumerate(procs):
                if codes[i] is None:
                    print(f"[bench] terminating rank {i} (pid {p.pid})", file=sys.stderr, flush=True)
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(0.2)
    return first_bad or next((c for c in codes if c), 0)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------
def build_index(n_tokens: int, vocab: int, seed: int, dev, corpus: str = "markov"):
    t0 = time.time()
    if corpus == "paq":
        text, beg = paq_corpus_gpu(n_tokens, vocab, seed, dev)
    else:
        text, beg = markov_corpus_gpu(n_tokens, vocab, seed, dev)
    torch.cuda.synchronize()
    t1 = time.time()
    log(f"corpus n={text.numel()} docs={beg.numel() - 1} in {t1 - t0:.1f}s; GPU construction ...")
    # fm_initialize_from_text_device: suffix array by GPU prefix doubling (64-bit
    # positions, csrc/sa.hip), SA / ISA samples for locate / extract, the index
    fm = FMIndex(device=dev.index)
    fm.initialize_from_text_device(text, keep_sa_text=True)
    torch.cuda.synchronize()
    t2 = time.time()
    bwt = fm.device_bwt()                  # the BWT: a copy materialised from E (stats: bwt_view_bytes)
    log(f"corpus {t1 - t0:.1f}s  suffix array + index {t2 - t1:.1f}s  n={bwt.numel()}")
    return fm, text, bwt, {"corpus_s": t1 - t0, "sa_and_index_s": t2 - t1, "beginnings": beg}


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


def lf_plan_bytes(prev_lo, prev_hi, tok, n, parent_cached, st, kernel: str):
    """Bytes the LF step of each row must read (64-B lines touched), mirroring
    lf_step_decode (fmidx_internal.h) and k_decode's workgroup E scan
    (decode.hip): full range -> C[c], C[c+1] + the C-block's cache id (2 lines);
    <= 512 rows -> E[lo, hi) (8 B per row); 513..kScanMax uncached rows
    (k_decode only) -> E[lo, hi); a range the transition table serves (a cached
    parent) -> its 16-slot probe (2 x 128 B) + the line of the parent's own cache
    entry, whose id the slots' keys hold (320 B); otherwise the 2-level wavelet-matrix
    descent: D2[c] + Z per level, and per level and endpoint the superblock
    count, the block header entry and the block prefix up to the position
    (level 0 exact from the position; level 1's position is data-dependent: its
    expected prefix, half a block).  Restarted / dead rows read nothing."""
    lo = np.asarray(prev_lo, dtype=np.int64)
    hi = np.minimum(np.asarray(prev_hi, dtype=np.int64), n)
    t = np.asarray(tok, dtype=np.int64)
    pc = np.asarray(parent_cached, dtype=bool)
    out = np.zeros(lo.size, dtype=np.int64)
    has_e = bool(st.get("lf_e", True))
    trans = st["trans_entries"] > 0
    cmin = st["cache_min"] or (1 << 62)
    scan_max = 4096 if kernel == "decode" and lo.size <= 256 else 1024
    w = hi - lo
    e_bytes = 64 * (((8 * hi + 63) // 64) - (8 * lo) // 64)   # 64-B lines of E[lo, hi)
    rest = (t >= 0) & (lo < hi)
    full = rest & (lo == 0) & (hi == n)
    out[full] = 128
    rest &= ~full
    if has_e:
        narrow = rest & (w <= 512)
        if kernel == "decode":
            narrow |= rest & (w <= scan_max) & ((w < cmin) | (not trans))
        out[narrow] = e_bytes[narrow]
        rest &= ~narrow
    probe = rest & trans & (w >= cmin)
    hit = probe & pc
    out[hit] = 320
    desc = rest & ~hit
    b = 320 * probe.astype(np.int64) + 3 * 64                # D2[c], Z[0][d0], Z[1][d1]
    for pos in (lo, hi):
        b = b + 2 * 64 + 64 * ((2 * (pos % 1024) + 63) // 64)  # level 0: sb + header + uint16 prefix
        b = b + 2 * 64 + 64 * ((512 + 63) // 64)             # level 1: sb + header + uint8 prefix (expected)
    out[desc] = b[desc]
    return out


def rank_pairs(fm, text, bwt, V, seed, dev, rows=65536, steps=9):
    """(tokens, lo, hi) of rows x (steps - 1) independent LF steps taken from
    a decode trace (the same generator as the bench's), plus the ranges the
    fused decode kernel computed for them (the exactness check)."""
    tokens, _, lo_h, hi_h, _ = decode_trace(fm, text, bwt, rows, V, steps, seed, dev)
    tok = tokens[1:steps].reshape(-1).contiguous()
    lo = lo_h[:steps - 1].reshape(-1).contiguous()
    hi = hi_h[:steps - 1].reshape(-1).contiguous()
    ref = (lo_h[1:steps].reshape(-1).contiguous(), hi_h[1:steps].reshape(-1).contiguous())
    return tok, lo, hi, ref


GATHER_MODES = {0: ("lane_64B", 1, 64), 2: ("coop4_64B", 4, 64), 3: ("coop8_128B", 8, 128), 4: ("lane_8B", 1, 8)}


def gather_ceiling(dev, nbytes=8 << 30):
    """The random-gather ceilings of HBM, measured live with
    csrc/probe.hip over an 8 GiB buffer: GB/s of independent random lines for
    each access shape (GATHER_MODES: every lane its own 64-B line, 4 lanes per
    64-B line, 8 lanes per 128-B line, every lane its own 8-B word -- bytes are
    the line bytes delivered), and ns per dependent hop with 256 chains (one
    chain per row at B = 256).  Returns (best 64-B-line ceiling, ns per hop,
    {mode: GB/s})."""
    buf = torch.randint(0, 1 << 62, (nbytes // 8,), dtype=torch.int64, device=dev)
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    threads, loads = 256 * 4096, 64
    rates = {}
    for mode, (name, lpl, line) in GATHER_MODES.items():
        best = None
        for _ in range(4):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            check(lib().fm_probe_gather(buf.data_ptr(), nbytes, mode, loads, threads, sink.data_ptr(), stream),
                  "probe")
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        rates[name] = threads // lpl * loads * line / (best * 1e-3) / 1e9
    gbs = max(rates["lane_64B"], rates["coop4_64B"])
    # the same shapes at the rank launch's size and temperature: ~1M requests
    # (2^19 pairs make ~1.07M) in ONE launch right after a 1 GiB eviction --
    # what a short cold gather kernel reaches, ramp and drain included
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    flush_acc = torch.zeros((), dtype=torch.int64, device=dev)
    for mode in (4, 3):
        name, lpl, line = GATHER_MODES[mode]
        thr = (1 << 20) * lpl // 8
        ts = []
        for _ in range(5):
            # enqueued behind the eviction while it runs (as the rank legs' timed() queued=True):
            # the events bracket the gather kernel, not the host's launch latency
            torch.cuda.synchronize()
            flush.add_(1)
            torch.sum(flush, 0, dtype=torch.int64, out=flush_acc)   # the rank legs' clean eviction
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            check(lib().fm_probe_gather(buf.data_ptr(), nbytes, mode, 8, thr, sink.data_ptr(), stream), "probe")
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        rates[name + "_1M_cold"] = thr // lpl * 8 * line / (float(np.median(ts)) * 1e-3) / 1e9
    del flush
    hops, chains = 4000, 256
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    check(lib().fm_probe_gather(buf.data_ptr(), nbytes, 1, hops, chains, sink.data_ptr(), stream), "probe")
    b.record()
    torch.cuda.synchronize()
    ns_hop = a.elapsed_time(b) * 1e6 / hops
    del buf
    torch.cuda.empty_cache()
    return gbs, ns_hop, rates


# ---------------------------------------------------------------------------
def cpu_share():
    """The CPUs this process is given, not the machine's: a shared GPU box shows
    every core of the host to os.cpu_count() / sched_getaffinity, while its CPU
    share is set by the cgroup quota and announced through OMP_NUM_THREADS.
    Returns (threads, where the number came from)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = f"sched_getaffinity {n}"
    try:                                   # cgroup v2: "quota period" or "max period"
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max" and int(per) > 0:
            c = max(1, -(-int(q) // int(per)))
            if c < n:
                n, src = c, f"cgroup cpu.max {q}/{per}"
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and 0 < int(env) < n:
        n, src = int(env), f"OMP_NUM_THREADS={env}"
    return n, src


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(fm, bwt, tokens, lo_hist, hi_hist, pats0, V, warmup, window, reps, dev):
    """The sdsl-faithful C++ restatement (oracle/cpu_ref.cpp) on the host
    cores, replaying the same trace, four legs: {incremental (one LF step per
    row per step, as the engine), full re-search (the reference's processors:
    get_count([last]), get_range(sent), get_count(sent) from scratch,
    document_constrained_generation_causal_qwen.py:97,135,138)} x {1 thread,
    every core this process may use}.  SURVEY §8(d): every leg times the SAME
    fixed window of `window` trace steps (steps warmup + 1 .. warmup + window),
    after one untimed warm-up step (step `warmup`: first touch of the index
    pages and the leg's buffers), `reps` times from the same state; the value
    is the median repetition (masks/s), with the min / max beside it.  Each
    leg's final ranges and final step's [B, V] masks are compared with the
    GPU's."""
    from oracle.cpu_ref import CpuRef

    t0 = time.time()
    ref = CpuRef.from_device_bwt(bwt)
    log(f"cpu_ref build {time.time() - t0:.1f}s")
    all_cores, share_src = cpu_share()
    B = tokens.shape[1]
    tok_np = tokens.cpu().numpy()
    lo_all = lo_hist.cpu().numpy().astype(np.uint64)
    hi_all = hi_hist.cpu().numpy().astype(np.uint64)
    first, last = warmup + 1, warmup + window           # the timed window, inclusive
    assert last < tokens.shape[0]
    # the full re-search legs' flat patterns per step (host bookkeeping, outside every timed region)
    pats = trace_patterns(pats0, tok_np, warmup - 1)
    flat_by_step = {}
    for s in range(warmup, last + 1):
        for b, t in enumerate(tok_np[s].tolist()):
            if t < 0:
                pats[b] = []
            else:
                pats[b].append(t)
        offs = np.zeros(B + 1, dtype=np.int64)
        np.cumsum([len(p) for p in pats], out=offs[1:])
        flat_by_step[s] = (np.fromiter((t for p in pats for t in p), dtype=np.int64), offs)

    dist_in_leg = []   # the incremental single-thread leg's own distinct_count time, per repetition

    def one_step(mode, s, lo, hi, mask, threads, acc=None):
        if mode == "incremental" and acc is not None:
            acc[0] += ref.decode_step_timed(np.ascontiguousarray(tok_np[s]), SHIFT, 0, lo, hi, mask)
        elif mode == "incremental":
            ref.decode_step(np.ascontiguousarray(tok_np[s]), SHIFT, 0, lo, hi, mask, threads)
        else:
            flat, offs = flat_by_step[s]
            ref.full_step(flat, offs, SHIFT, lo, hi, mask, threads, faithful=True)

    # every leg: one untimed warm-up step, then `reps` timed passes over the same window; the
    # repetitions are interleaved across the legs (A B C D A B C D ...), so drift of the shared
    # host (frequency, other tenants) lands on every leg alike
    names = [(mode, threads) for mode in ("incremental", "full_research") for threads in (1, all_cores)]
    state = {}
    for mode, threads in names:
        mask = np.zeros((B, V), dtype=np.uint8)
        lo = lo_all[warmup - 1].copy()
        hi = hi_all[warmup - 1].copy()
        one_step(mode, warmup, lo, hi, mask, threads)          # untimed warm-up step
        state[(mode, threads)] = (lo, hi, mask, lo.copy(), hi.copy(), [])
    # the part of a single-thread step that is distinct_count (fm_index.cpp:119-144: three
    # sigma-sized zeroed vectors + the interval_symbols DFS): the same window's ranges -- the ones
    # each step's LF produced, which the incremental leg enumerates -- timed as a fifth leg in the
    # same interleaving, so it is a part of the same work as the whole steps it is compared with
    ref.distinct_only(lo_all[warmup], hi_all[warmup], 1)       # untimed warm-up, like the legs
    dts = []
    for _ in range(reps):
        for key in names:
            lo, hi, mask, lo_w, hi_w, rates = state[key]
            lo[:] = lo_w
            hi[:] = hi_w
            acc = [0.0] if key == ("incremental", 1) else None
            a = time.perf_counter()
            for s in range(first, last + 1):
                one_step(key[0], s, lo, hi, mask, key[1], acc)
            rates.append(window * B / (time.perf_counter() - a))
            if acc is not None:
                dist_in_leg.append((acc[0] / window, B / rates[-1]))
        a = time.perf_counter()
        for s in range(first, last + 1):
            ref.distinct_only(lo_all[s], hi_all[s], 1)
        dts.append((time.perf_counter() - a) / window)
        # one line per repetition: a long CPU leg must not look like a hung run
        log(f"cpu repetition {len(dts)}/{reps}: " +
            ", ".join(f"{m}x{t} {state[(m, t)][5][-1]:.0f}" for m, t in names) + " masks/s")
    legs = {}
    for (mode, threads), (lo, hi, mask, _, _, rates) in state.items():
        ok = bool(np.array_equal(lo, lo_all[last]) and np.array_equal(hi, hi_all[last]))
        gmask = fm.allowed_mask(lo_hist[last], hi_hist[last], V, SHIFT).cpu().numpy()
        mok = bool(np.array_equal(mask, gmask))
        med = float(np.median(rates))
        legs[f"{mode}_{'1' if threads == 1 else 'all'}"] = {
            "value": med, "min": float(min(rates)), "max": float(max(rates)),
            "spread": float((max(rates) - min(rates)) / med), "reps": reps, "threads": threads,
            "steps": window, "ranges_match_gpu": ok, "masks_match_gpu": mok}
        log(f"cpu {mode} x{threads}: median {med:.0f} masks/s ({min(rates):.0f}-{max(rates):.0f}) over "
            f"{reps} x {window} steps; ranges ok {ok}, masks ok {mok}")
    per_step = {"distinct_count_only": float(np.median(dts)),
                "incremental": B / legs["incremental_1"]["value"],
                "full_research": B / legs["full_research_1"]["value"],
                # measured inside the incremental single-thread leg's own steps (a part of the same run,
                # per repetition): it cannot exceed that leg's step
                "distinct_count_in_incremental": float(np.median([d for d, _ in dist_in_leg])),
                "distinct_count_share_of_incremental": float(np.median([d / w for d, w in dist_in_leg]))}
    log(f"cpu 1-thread seconds per step: {per_step}")
    head = legs["incremental_all"]
    return {"value": head["value"], "unit": "masks/s", "cores": all_cores, "kind": "port",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "cores_source": share_src,
            "sample": f"trace steps {first}..{last} ({window} steps x {B} rows) of the same trace and "
                      f"n={bwt.numel()} index, after one untimed warm-up step, median of {reps} repetitions; "
                      f"sdsl-faithful wt_int + rank_support_v restatement (oracle/cpu_ref.cpp); value = the "
                      f"incremental leg on the {all_cores} cores this process is given ({share_src}; the "
                      f"fastest CPU mode); the reference's own per-step work is the full_research legs",
            "legs": legs,
            "one_thread_s_per_step": per_step,
            "ranges_match_gpu": all(v["ranges_match_gpu"] for v in legs.values()),
            "masks_match_gpu": all(v["masks_match_gpu"] for v in legs.values())}


# ---------------------------------------------------------------------------
def mem_log(tag, dev):
    free, total = torch.cuda.mem_get_info(dev)
    log(f"[mem] {tag}: {free / 2**30:.1f} GiB free of {total / 2**30:.1f}")


def shard_trace(fm, text, bwt, B, V, S, dev):
    """The trace every rank of the sharded mode decodes (the same rows on every
    rank: seeded identically), taken from the replica while it and the corpus
    are resident, with the replica's uint8 masks of the last step (the
    exactness reference).  Computing it here lets the legs free the replica
    before they regenerate the corpus (replica + corpus + a build would not fit
    in HBM together at C3)."""
    tokens, _, lo_hist, hi_hist, pats0 = decode_trace(fm, text, bwt, B, V, S, 777, dev)
    ref = fm.allowed_mask(lo_hist[S - 1], hi_hist[S - 1], V, SHIFT)
    return tokens, pats0, ref


def sharded_leg(holder, text_seed, n_tokens, V, K, W, world, rank, dev, shs, halo=128):
    """Doc-range sharded decode, measured after the
    replica run at N > 1.  The traces (tokens + initial patterns, one per
    global batch size in ``shs``: the metric's B = 256 and the PAQ eval shape's
    2048 rows) and the reference masks of their last step come from the replica
    (unsharded) index; then every rank indexes its doc range + halo (one slice
    of T', built on the device, once) and decodes all B rows against it.  A
    step is the fused LF + mask, then the exchange:
    "dense" -- RCCL all_gather of every row's packed bitmap and fm_or_bits;
    "sparse" -- fm_shard_pack (per row the shard's BWT slice when smaller than
    the bitmap, else the bitmap), an all_gather of the payload sizes (read on
    the host), an all_gather of the payloads and ONE fused OR / scatter /
    unpack pass (fm_shard_or_rows); "peer" -- the decode kernel writes the
    payload into IPC-mapped buffers, a one-element RCCL all_reduce as the
    stream-ordered barrier, and the OR pass reading every rank's payload in
    place over xGMI (fm_shard_or_rows_peers); "peer_flags" -- the same with
    the flag barrier (device step counter, fm_peer_signal + the polling OR
    pass): no collective in the step; "peer_flags_graph" -- that step captured
    ONCE into a HIP graph and replayed K times (each replay after a copy of
    the step's tokens into the graph's static input), the serving loop's form.
    Each mode is timed over the same K steps and its last step's mask must
    equal the replica's; ``value`` is the fastest exact mode at B = 256.
    FMIDX_BENCH_PEER=0 leaves the peer modes out."""
    import torch.distributed as dist

    from fmidx.sharding import PeerExchange, SparseExchange, or_bits, shard_text_device, unpack_bits

    fm, bwt = holder.pop(), holder.pop()      # the replica index and its BWT (the caller keeps no reference)
    S = W + K
    del bwt, fm
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    t0 = time.time()
    ix, err = None, ""
    try:
        text, beg = markov_corpus_gpu(n_tokens, V, text_seed, dev)
        shard, (a, b) = shard_text_device(text, beg, world, rank, halo)
        del text
        torch.cuda.empty_cache()
        ix = FMIndex(device=dev.index)
        ix.initialize_from_text_device(shard)
        del shard
        torch.cuda.synchronize()
    except Exception as e:   # every rank learns of it below: no rank is left waiting in a collective
        err = repr(e)
    build_s = time.time() - t0
    ok_all = torch.tensor([0 if err else 1], device=dev)
    dist.all_reduce(ok_all, op=dist.ReduceOp.MIN)
    if not int(ok_all.item()):
        raise RuntimeError(f"shard build failed on some rank ({err or 'another rank'})")
    Bmax = max(shs)
    Wd = (V + 31) // 32
    peer, peer_err = None, ""
    if os.environ.get("FMIDX_BENCH_PEER", "1") != "0":
        try:
            peer = PeerExchange(None, Bmax, V, dev, barrier="collective")
        except Exception as e:   # every rank learns of it below
            peer_err = repr(e)
        ok_all = torch.tensor([0 if peer_err else 1], device=dev)
        dist.all_reduce(ok_all, op=dist.ReduceOp.MIN)
        if not int(ok_all.item()):
            if peer is not None:
                peer.close()
            peer, peer_err = None, peer_err or "the peer mapping failed on another rank"

    def one_batch(B, tokens, pats0, ref):
        lens = [len(p) for p in pats0]
        assert max(lens) + S <= halo - 1, "trace patterns would outgrow the halo"
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), device=dev)
        toks = torch.tensor([t for p in pats0 for t in p], dtype=torch.int64, device=dev)
        lo0 = torch.zeros(B, dtype=torch.int64, device=dev)
        hi0 = torch.zeros(B, dtype=torch.int64, device=dev)
        ix.backward_search_batch(toks, offs, SHIFT, lo0, hi0)
        mine = torch.empty((B, Wd), dtype=torch.int32, device=dev)
        parts = torch.empty((world, B, Wd), dtype=torch.int32, device=dev)
        out = torch.empty((B, V), dtype=torch.uint8, device=dev)
        outw = torch.empty((B, Wd), dtype=torch.int32, device=dev)
        payload = None
        words_seen = []
        xchg = SparseExchange(None)

        def run(mode):
            nonlocal payload
            lo, hi = lo0.clone(), hi0.clone()
            bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]
            flags = mode in ("peer_flags", "peer_flags_graph", "peer_flags_checked", "peer_flags_packed")
            checked = mode == "peer_flags_checked"
            packed_out = mode == "peer_flags_packed"
            tok_static = torch.empty_like(tokens[0])

            def step(i, tok=None):
                nonlocal payload
                src, dst = bufs[i % 2], bufs[(i + 1) % 2]
                if flags:            # state in place, the buffer and the step number on the device
                    # one C call (fm_peer_flags_step, as ShardedDecoder makes it); checked: it also
                    # synchronises the stream, then the error word is read -- exact or absent
                    peer.flags_step(ix, tokens[i] if tok is None else tok, lo, hi, V, SHIFT,
                                    outw if packed_out else out, unpack=not packed_out, sync=checked)
                    if checked:
                        peer.check()
                    return
                if mode == "peer":   # the decode kernel writes the payload itself
                    pay = peer.payload()
                    ix.decode_step_payload(tokens[i], src[0], src[1], dst[0], dst[1], pay, V, SHIFT, reset_below=0)
                    peer(pay, B, V, SHIFT, out=out)
                    return
                ix.decode_step(tokens[i], src[0], src[1], mine, V, SHIFT, reset_below=0, lo_out=dst[0],
                               hi_out=dst[1], packed=True)
                if mode == "dense":
                    dist.all_gather_into_tensor(parts, mine)
                    or_bits(parts, V, out=out)
                else:
                    payload = ix.shard_pack(dst[0], dst[1], mine, V, payload=payload)
                    xchg(payload, B, V, SHIFT, out=out)
                    if i >= W:
                        words_seen.append(xchg.words[-1])

            peer_mode = mode in ("peer", "peer_flags", "peer_flags_graph")
            if peer_mode:
                peer.barrier_mode = "flags" if flags else "collective"
            for i in range(W):
                step(i)
            g = None
            if mode == "peer_flags_graph":
                # ONE step captured (no collective in it: the flag words over xGMI, the step number
                # on the device), replayed for every timed step after its tokens are copied in
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    step(W, tok_static)
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
            a_ev = torch.cuda.Event(enable_timing=True)
            b_ev = torch.cuda.Event(enable_timing=True)
            a_ev.record()
            for i in range(W, S):
                if g is not None:
                    tok_static.copy_(tokens[i])
                    g.replay()
                else:
                    step(i)
            b_ev.record()
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()
            t = torch.tensor([a_ev.elapsed_time(b_ev) / K], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if packed_out:           # the ORed words, expanded outside the timed region for the check
                exact = bool(torch.equal(unpack_bits(outw.view(torch.uint8), V), ref))
            else:
                exact = bool(torch.equal(out, ref))
            timeouts = 0
            if flags:
                timeouts = peer.errors()
            ok = torch.tensor([1 if exact and not timeouts else 0], device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            return float(t.item()), bool(ok.item()), timeouts

        ms_dense, exact_dense, _ = run("dense")
        ms_sparse, exact_sparse, _ = run("sparse")
        per_step = [sum(w) for w in words_seen]
        modes = {
            "dense": {"ms_per_step": ms_dense, "value": B / (ms_dense / 1e3), "masks_equal_unsharded": exact_dense,
                      "exchange_bytes_per_step": world * B * Wd * 4,
                      "step": "RCCL all_gather of the packed rows + fm_or_bits"},
            "sparse": {"ms_per_step": ms_sparse, "value": B / (ms_sparse / 1e3),
                       "masks_equal_unsharded": exact_sparse,
                       "exchange_bytes_per_step_median": 4.0 * float(np.median(per_step)) if per_step else None,
                       "speculative_gathers_respecified": xchg.respecified,
                       "allgather_bytes_per_step_median": (4.0 * world * float(np.median([max(w) for w in words_seen]))
                                                           if words_seen else None),
                       "step": "fm_shard_pack, all_gather of sizes (host read) + payloads, fm_shard_or_rows"},
        }
        if peer is not None:
            ms_peer, exact_peer, _ = run("peer")
            modes["peer"] = {"ms_per_step": ms_peer, "value": B / (ms_peer / 1e3), "masks_equal_unsharded": exact_peer,
                             "exchange_bytes_per_step_median": modes["sparse"]["exchange_bytes_per_step_median"],
                             "step": "fm_decode_step_payload (the decode kernel writes the payload, fixed row "
                                     "slots) into IPC-mapped buffers, 1-element RCCL all_reduce (barrier), "
                                     "fm_shard_or_rows_peers reading every rank's payload over xGMI"}
            ms_pf, exact_pf, to_pf = run("peer_flags")
            modes["peer_flags"] = {"ms_per_step": ms_pf, "value": B / (ms_pf / 1e3),
                                   "masks_equal_unsharded": exact_pf, "flag_timeouts": to_pf,
                                   "step": "as peer, with the flag barrier, one C call per step (fm_peer_flags_step): "
                                           "the payload decode with the signal fused into its last workgroup (the "
                                           "device step counter advanced, a system-scope release, stores into every "
                                           "rank's flag array) + fm_shard_or_rows_peers_wait; state updated in place; "
                                           "eager launches; the error word read only after the timed region "
                                           "(ShardedDecoder's check='deferred')"}
            ms_pp, exact_pp, to_pp = run("peer_flags_packed")
            modes["peer_flags_packed"] = {"ms_per_step": ms_pp, "value": B / (ms_pp / 1e3),
                                          "masks_equal_unsharded": exact_pp, "flag_timeouts": to_pp,
                                          "output": "packed int32 [B, ceil(V/32)] words (bit t = token t)",
                                          "step": "as peer_flags with the OR pass writing the packed words "
                                                  "(ShardedDecoder(unpack=False), what the processors' epilogue "
                                                  "reads) instead of the uint8 mask: V/8 bytes per row, not V"}
            ms_pc, exact_pc, to_pc = run("peer_flags_checked")
            modes["peer_flags_checked"] = {"ms_per_step": ms_pc, "value": B / (ms_pc / 1e3),
                                           "masks_equal_unsharded": exact_pc, "flag_timeouts": to_pc,
                                           "wait_cost_us_per_step": (ms_pc - ms_pf) * 1e3,
                                           "step": "as peer_flags, plus the exact-or-absent check every step "
                                                   "(ShardedDecoder's default check='sync'): the same C call "
                                                   "synchronises the stream after the OR pass, then the error "
                                                   "word is read"}
            try:
                ms_pg, exact_pg, to_pg = run("peer_flags_graph")
                modes["peer_flags_graph"] = {"ms_per_step": ms_pg, "value": B / (ms_pg / 1e3),
                                             "masks_equal_unsharded": exact_pg, "flag_timeouts": to_pg,
                                             "step": "peer_flags captured ONCE as a one-step HIP graph, replayed K "
                                                     "times (tokens copied into its static input before each "
                                                     "replay): the per-token serving loop"}
            except Exception as e:   # capture refused: the eager figures stand
                modes["peer_flags_graph"] = {"value": None, "error": repr(e)}
        else:
            modes["peer"] = {"value": None, "error": peer_err or "disabled (FMIDX_BENCH_PEER=0, or the "
                                                                      "peer preflight was not exact on every rank)"}
        # the headline sharded figure is a uint8 mask like the replica's; the packed-output mode is reported beside it
        exact_modes = [m for m, r in modes.items() if r.get("masks_equal_unsharded") and m != "peer_flags_packed"]
        best = min(exact_modes, key=lambda m: modes[m]["ms_per_step"]) if exact_modes else "sparse"
        return {"value": modes[best]["value"], "ms_per_step": modes[best]["ms_per_step"], "global_batch": B,
                "masks_equal_unsharded": bool(exact_modes) and modes[best]["masks_equal_unsharded"],
                "exchange": best, "modes": modes}

    by_batch = {}
    for B in sorted(shs):
        tokens, pats0, ref = shs[B]
        by_batch[B] = one_batch(B, tokens, pats0, ref)
        log(f"sharded B={B}: {by_batch[B]['value'] / 1e6:.2f} M masks/s ({by_batch[B]['exchange']}, "
            f"{by_batch[B]['ms_per_step'] * 1e3:.1f} us/step), exact {by_batch[B]['masks_equal_unsharded']}")
    if peer is not None:
        peer.close()
    head = by_batch[256] if 256 in by_batch else by_batch[min(by_batch)]
    st = ix.stats()
    return {"metric": "allowed-token masks/sec (doc-range sharded, C4)", "value": head["value"],
            "unit": "masks/s", "ms_per_step": head["ms_per_step"], "scaling": "strong", "shards": world,
            "halo": halo, "global_batch": head["global_batch"], "shard_docs": [int(a), int(b)],
            "shard_rows": ix.size(), "shard_device_bytes": st["device_bytes"], "shard_build_s": build_s,
            "masks_equal_unsharded": head["masks_equal_unsharded"], "exchange": head["exchange"],
            "modes": head["modes"], "by_global_batch": {str(k): v for k, v in by_batch.items()},
            "payload": "per row the shard's BWT slice (hi - lo < ceil(V/32)) or its packed bitmap",
            "step": "fused LF + mask, then the exchange of 'exchange' (modes: each timed over the same K steps), "
                    "uint8 [B, V] out"}


def after_replica_legs(holder, text_seed, n_tokens, V, B, K, W, dev, main_trace, sh, world=8, halo=128):
    """Legs that need the replica index gone (N = 1, C3): the compact memory
    profile of the same corpus, then C4 on one GPU.  Returns
    (compact, c4) result dicts.

    Compact: the index rebuilt with the compact build profile (fm_build_options
    FM_PROFILE_COMPACT: transitions to cached children only, no E array, no
    probe-first) -- the same BWT, so the headline trace's K
    steps replay from the same state and must end in the same ranges; timed
    cold like the headline.

    C4 (the corpus doc-range sharded 8 ways) rehearsed on ONE
    GPU: the 8 shards are built one after another, each decodes the B rows of
    the replica's trace with its K timed steps captured in a HIP graph (cold
    replay after a 1 GiB eviction, as the headline), writing bit-packed rows --
    the per-rank kernel work of the 8-GPU run at n/8 rows -- and the OR of the
    8 shards' last-step rows (fm_or_bits, the only post-exchange pass) is timed
    the same way and checked against the replica's uint8 mask.  The exchange
    itself (all_gather of 8 x B x V/8 bytes over xGMI) cannot run on one GPU;
    ``predicted_step_us`` adds a stated model of it."""
    from fmidx.sharding import or_bits, or_payloads, or_peer_payloads, payload_capacity, shard_text_device

    fm, bwt = holder.pop(), holder.pop()
    S = W + K
    tokens, pats0, ref = sh                   # shard_trace, taken while the replica was resident
    del bwt, fm
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    mem_log(f"replica freed (torch reserves {torch.cuda.memory_reserved(dev) / 2**30:.1f} GiB)", dev)
    text, beg = markov_corpus_gpu(n_tokens, V, text_seed, dev)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)

    def replay(g, cold):
        if cold:
            flush.add_(1)
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b)

    # ---- the compact memory profile, same corpus and trace as the headline
    compact = {}
    try:
        m_tok, m_lo, m_hi, f_lo, f_hi = main_trace
        t0 = time.time()
        cx = FMIndex(device=dev.index, options="compact")
        cx.initialize_from_text_device(text)
        torch.cuda.synchronize()
        cbuild = time.time() - t0
        mask = torch.empty((B, V), dtype=torch.uint8, device=dev)
        lo, hi = m_lo.clone(), m_hi.clone()
        bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(K):
                src, dst = bufs[i % 2], bufs[(i + 1) % 2]
                cx.decode_step(m_tok[i], src[0], src[1], mask, V, SHIFT, reset_below=0, lo_out=dst[0], hi_out=dst[1])
        warm = []
        for _ in range(3):
            lo.copy_(m_lo)
            hi.copy_(m_hi)
            warm.append(replay(g, False) / K * 1e3)
        lo.copy_(m_lo)
        hi.copy_(m_hi)
        cold = replay(g, True) / K * 1e3
        fin = bufs[K % 2]
        cst = cx.stats()
        compact = {"build_options": cx.build_options(), "device_bytes": int(cst["device_bytes"]),
                   "build_s": round(cbuild, 1),
                   "cold_ms_per_step": cold / 1e3, "warm_ms_per_step": float(np.median(warm)) / 1e3,
                   "value_cold": B / (cold * 1e-6),
                   "ranges_equal_default_profile": bool(torch.equal(fin[0], f_lo) and torch.equal(fin[1], f_hi))}
        log(f"compact profile: {cst['device_bytes'] / 2**30:.1f} GiB, step cold {cold:.1f}us warm {np.median(warm):.1f}us, "
            f"exact {compact['ranges_equal_default_profile']}")
        del g, cx, bufs, lo, hi, mask
        torch.cuda.empty_cache()
    except Exception as e:      # the C4 leg and the line still run
        compact = {"error": repr(e), "where": traceback.format_exc()[-1200:]}

    def c4_part():
        lens = [len(p) for p in pats0]
        assert max(lens) + S <= halo - 1, "trace patterns would outgrow the halo"
        offs = torch.tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64), device=dev)
        toks = torch.tensor([t for p in pats0 for t in p], dtype=torch.int64, device=dev)
        Wd = (V + 31) // 32
        parts = torch.empty((world, B, Wd), dtype=torch.int32, device=dev)
        shards, last_pay, pay_words, fix_pay = [], [], [], []
        for r in range(world):
            t0 = time.time()
            t_r, (a, b) = shard_text_device(text, beg, world, r, halo)
            ix = FMIndex(device=dev.index)
            ix.initialize_from_text_device(t_r)
            rows = t_r.numel()
            del t_r
            torch.cuda.synchronize()
            build_s = time.time() - t0
            lo = torch.zeros(B, dtype=torch.int64, device=dev)
            hi = torch.zeros(B, dtype=torch.int64, device=dev)
            ix.backward_search_batch(toks, offs, SHIFT, lo, hi)
            lo[1], hi[1] = 0, 0                    # the trace's eos row (its pattern ends with an unknown id)
            for i in range(W):
                ix.decode_step(tokens[i], lo, hi, parts[r], V, SHIFT, reset_below=0, packed=True)
            s_lo, s_hi = lo.clone(), hi.clone()
            bufs = [(lo, hi), (torch.empty_like(lo), torch.empty_like(hi))]
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(K):
                    src, dst = bufs[i % 2], bufs[(i + 1) % 2]
                    ix.decode_step(tokens[W + i], src[0], src[1], parts[r], V, SHIFT, reset_below=0,
                                   lo_out=dst[0], hi_out=dst[1], packed=True)
            warm = []
            for _ in range(3):
                lo.copy_(s_lo)
                hi.copy_(s_hi)
                warm.append(replay(g, False) / K * 1e3)
            lo.copy_(s_lo)
            hi.copy_(s_hi)
            cold = replay(g, True) / K * 1e3          # leaves parts[r] = this shard's last-step rows
            fin_lo, fin_hi = bufs[K % 2][0].clone(), bufs[K % 2][1].clone()
            # sparse exchange: this shard's payload of every timed step (sizes), the last one kept
            pay = ix.shard_pack(fin_lo, fin_hi, parts[r], V)
            g_pack = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_pack):
                for _ in range(K):
                    ix.shard_pack(fin_lo, fin_hi, parts[r], V, payload=pay)
            pack_cold = replay(g_pack, True) / K * 1e3
            last_pay.append(pay[:int(pay[0].item())].clone())
            lo.copy_(s_lo)
            hi.copy_(s_hi)
            scratch = torch.empty_like(parts[r])
            sizes = []
            for i in range(K):
                src, dst = bufs[i % 2], bufs[(i + 1) % 2]
                ix.decode_step(tokens[W + i], src[0], src[1], scratch, V, SHIFT, reset_below=0,
                               lo_out=dst[0], hi_out=dst[1], packed=True)
                sizes.append(int(ix.shard_pack(dst[0], dst[1], scratch, V, payload=pay)[0].item()))
            pay_words.append(sizes)
            del g_pack, pay, scratch
            # the peer exchange's decode: the kernel writes the payload itself (fixed row slots, no pack);
            # the same K steps from the same state, graph-captured, cold like the packed steps
            fpay = torch.zeros(payload_capacity(B, V), dtype=torch.int32, device=dev)
            g_pd = torch.cuda.CUDAGraph()
            lo.copy_(s_lo)
            hi.copy_(s_hi)
            with torch.cuda.graph(g_pd):
                for i in range(K):
                    src, dst = bufs[i % 2], bufs[(i + 1) % 2]
                    ix.decode_step_payload(tokens[W + i], src[0], src[1], dst[0], dst[1], fpay, V, SHIFT,
                                           reset_below=0)
            pd_warm = []
            for _ in range(3):
                lo.copy_(s_lo)
                hi.copy_(s_hi)
                pd_warm.append(replay(g_pd, False) / K * 1e3)
            lo.copy_(s_lo)
            hi.copy_(s_hi)
            pd_cold = replay(g_pd, True) / K * 1e3
            pd_same = bool(torch.equal(bufs[K % 2][0], fin_lo) and torch.equal(bufs[K % 2][1], fin_hi))
            fix_pay.append(fpay)
            del g_pd
            st = ix.stats()
            shards.append({"docs": [int(a), int(b)], "rows": int(rows), "device_bytes": int(st["device_bytes"]),
                           "build_s": round(build_s, 2), "cold_us_per_step": cold,
                           "warm_us_per_step": float(np.median(warm)), "pack_cold_us": pack_cold,
                           "payload_bytes_per_step_median": 4.0 * float(np.median(sizes)),
                           "payload_decode_cold_us": pd_cold, "payload_decode_warm_us": float(np.median(pd_warm)),
                           "payload_decode_states_equal": pd_same})
            mem_log(f"c4 shard {r} built", dev)
            log(f"c4 shard {r}: rows {rows}, build {build_s:.1f}s, step cold {cold:.1f}us warm {np.median(warm):.1f}us")
            del g, ix, bufs, lo, hi, s_lo, s_hi
            torch.cuda.empty_cache()
        out = torch.empty((B, V), dtype=torch.uint8, device=dev)
        or_bits(parts, V, out=out)
        exact = bool(torch.equal(out, ref))
        # the OR pass timed like the steps: K launches in one graph (one launch alone is
        # mostly graph-launch overhead), each over its own copy of the gathered rows --
        # K x 33 MB, beyond the MALL -- so that after the eviction every launch reads cold
        pk = parts.unsqueeze(0).expand(K, *parts.shape).contiguous()
        g_or = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_or):
            for i in range(K):
                or_bits(pk[i], V, out=out)
        or_warm = float(np.median([replay(g_or, False) for _ in range(3)])) / K * 1e3
        or_cold = replay(g_or, True) / K * 1e3
        exact = exact and bool(torch.equal(out, ref))
        del pk, g_or
        # the sparse exchange's OR / scatter / unpack over the 8 last-step payloads (padded to the
        # largest, as the all_gather delivers them), timed the same way
        m = max(p.numel() for p in last_pay)
        sp = torch.zeros((world, m), dtype=torch.int32, device=dev)
        for r, p in enumerate(last_pay):
            sp[r, :p.numel()] = p
        out.zero_()
        or_payloads(sp, B, V, SHIFT, out=out)
        exact_sparse = bool(torch.equal(out, ref))
        spk = sp.unsqueeze(0).expand(K, *sp.shape).contiguous()
        g_sp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_sp):
            for i in range(K):
                or_payloads(spk[i], B, V, SHIFT, out=out)
        sp_warm = float(np.median([replay(g_sp, False) for _ in range(3)])) / K * 1e3
        sp_cold = replay(g_sp, True) / K * 1e3
        exact_sparse = exact_sparse and bool(torch.equal(out, ref))
        del spk, g_sp, sp
        # the peer exchange's pass (fm_shard_or_rows_peers) over the 8 shards' last-step payloads as the
        # payload decode wrote them (fixed row slots, each in a buffer of its own, as the ranks'
        # IPC-mapped buffers are -- here local)
        cap = payload_capacity(B, V)
        pb = torch.zeros((K, world, cap), dtype=torch.int32, device=dev)
        for r, p in enumerate(fix_pay):
            pb[:, r, :p.numel()] = p
        ptabs = torch.tensor([[pb[i, r].data_ptr() for r in range(world)] for i in range(K)], dtype=torch.int64,
                             device=dev)
        out.zero_()
        or_peer_payloads(ptabs[0], cap, B, V, SHIFT, out=out)
        exact_peer = bool(torch.equal(out, ref))
        g_pp = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_pp):
            for i in range(K):
                or_peer_payloads(ptabs[i], cap, B, V, SHIFT, out=out)
        pp_warm = float(np.median([replay(g_pp, False) for _ in range(3)])) / K * 1e3
        pp_cold = replay(g_pp, True) / K * 1e3
        exact_peer = exact_peer and bool(torch.equal(out, ref))
        del pb, ptabs, g_pp
        step_words = [sum(w[i] for w in pay_words) for i in range(K)]
        step_max = [max(w[i] for w in pay_words) for i in range(K)]
        # exchange model: every rank receives (world - 1) packed slices of B x 4 ceil(V/32)
        # bytes over its 7 point-to-point xGMI links (~153 GB/s each, direct: one slice per
        # link in parallel) plus a ~15 us collective latency; a ring (one link, 7 hops) is the
        # pessimistic bound.  The driver's 8-GPU run measures the real figure.
        slice_b = B * Wd * 4
        ag_direct = slice_b / 153e9 * 1e6 + 15.0
        ag_ring = (world - 1) * slice_b / 153e9 * 1e6 + 15.0
        slow = max(s["cold_us_per_step"] for s in shards)
        pack = max(s["pack_cold_us"] for s in shards)
        sp_slice = 4.0 * float(np.median(step_max))          # the largest rank's payload: what every link carries
        ag_sp_direct = sp_slice / 153e9 * 1e6 + 15.0
        ag_sp_ring = (world - 1) * sp_slice / 153e9 * 1e6 + 15.0
        sizes_us = 15.0                                       # the all_gather of the sizes + the host read
        sparse = {"masks_equal_unsharded": exact_sparse, "or_rows_cold_us": sp_cold, "or_rows_warm_us": sp_warm,
                  "pack_cold_us_slowest_shard": pack,
                  "payload_bytes_per_step_all_ranks_median": 4.0 * float(np.median(step_words)),
                  "payload_bytes_per_step_largest_rank_median": sp_slice,
                  "dense_bytes_per_step_all_ranks": world * slice_b,
                  "allgather_model_us": {"direct_7_links": ag_sp_direct, "ring": ag_sp_ring,
                                         "sizes_exchange_us_assumed": sizes_us},
                  "predicted_step_us": {"direct": slow + pack + sizes_us + ag_sp_direct + sp_cold,
                                        "ring": slow + pack + sizes_us + ag_sp_ring + sp_cold},
                  "note": "per row the shard's BWT slice when hi - lo < ceil(V/32), else its bitmap "
                          "(fm_shard_pack); OR / scatter / unpack of the 8 payloads (fm_shard_or_rows)"}
        # peer model: the same pack; a one-element all_reduce as the barrier (assumed 15 us at 8
        # ranks); the OR pass reads the 7 peers' payloads over the 7 links in parallel (the largest
        # payload / 153 GB/s on top of the pass measured here over local buffers, + 2 us per remote
        # round trip: the header, then the data)
        remote_us = sp_slice / 153e9 * 1e6 + 2 * 2.0
        slow_pd = max(s["payload_decode_cold_us"] for s in shards)
        peer = {"masks_equal_unsharded": exact_peer, "or_rows_peers_cold_us": pp_cold,
                "or_rows_peers_warm_us": pp_warm, "payload_decode_cold_us_slowest_shard": slow_pd,
                "payload_decode_states_equal": all(s["payload_decode_states_equal"] for s in shards),
                "barrier_us_assumed": 15.0, "remote_read_model_us": remote_us,
                "predicted_step_us": slow_pd + 15.0 + remote_us + pp_cold,
                # the flag barrier instead of the all_reduce: one xGMI store + the poll that sees it
                "flag_barrier_us_assumed": 3.0,
                "predicted_step_us_flags": slow_pd + 3.0 + remote_us + pp_cold,
                "note": "the decode kernel writes each shard's payload (fixed row slots, no pack pass) into "
                        "IPC-mapped buffers read in place (fm_shard_or_rows_peers): no sizes exchange, no "
                        "gather; here over local buffers"}
        return {"shards": world, "halo": halo, "global_batch": B, "steps": K, "per_shard": shards,
                "sparse_exchange": sparse, "peer_exchange": peer,
                "slowest_shard_cold_us": slow, "or_pass_cold_us": or_cold, "or_pass_warm_us": or_warm,
                "or_pass_bytes": world * slice_b + B * V,
                "or_pass_GBps_cold": (world * slice_b + B * V) / (or_cold * 1e-6) / 1e9,
                "or_pass_timing": f"{K} launches in one graph, each over its own copy of the gathered rows, / {K}",
                "masks_equal_unsharded": exact,
                "allgather_model_us": {"direct_7_links": ag_direct, "ring": ag_ring,
                                       "slice_bytes": slice_b, "link_GBps_assumed": 153.0, "latency_us_assumed": 15.0},
                "predicted_step_us": {"direct": slow + ag_direct + or_cold, "ring": slow + ag_ring + or_cold},
                "note": "one GPU: shards built and timed in turn (graph-captured K steps, cold), packed rows of all 8 "
                        "ORed by fm_or_bits and compared with the replica's uint8 mask of the same step"}

    try:
        return compact, c4_part()
    except Exception as e:      # the compact result still reaches the line
        return compact, {"error": repr(e), "where": traceback.format_exc()[-1200:]}


# ---------------------------------------------------------------------------
# The peer exchange's cross-device preflight (N > 1).  The sharded leg's peer modes are the first
# code here to map another GPU's memory (hipIpc), store flag words over xGMI and read payloads in
# place with system-scope loads; a GPU fault there would end the rank's process before its
# measured line is printed.  So each rank first runs those mechanics in a CHILD process on a tiny
# corpus: a fault ends the child only, and the ranks then skip the peer modes (dense and sparse
# still run) with the reason in the line.
PREFLIGHT_PORT_OFFSET = 101   # the children's gloo rendezvous: MASTER_PORT + this
PREFLIGHT_TIMEOUT_S = 180.0


def peer_preflight_child() -> int:
    """``bench.py --peer-preflight``: ShardedDecoder(reduce="peer", the flag barrier, check="sync")
    over 6 steps of a 400-doc corpus sharded WORLD_SIZE ways, against the unsharded decoder, on
    device LOCAL_RANK (FMIDX_PREFLIGHT_DEVICE overrides it: the one-GPU test runs both ranks on
    device 0).  The group is gloo on 127.0.0.1:FMIDX_PREFLIGHT_PORT (the IPC handles' exchange;
    no RCCL communicator).  Returns the exit status: 0 exact, 1 inexact or an exception."""
    import datetime

    import torch.distributed as dist

    from fmidx.index import FMIndex as DocIndex
    from fmidx.sharding import ShardedDecoder, shard_corpus

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    d = int(os.environ.get("FMIDX_PREFLIGHT_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(d)
    dev = torch.device("cuda", d)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{int(os.environ['FMIDX_PREFLIGHT_PORT'])}",
                            world_size=world, rank=rank, timeout=datetime.timedelta(seconds=120))
    ok = False
    try:
        V, halo, B = 128256, 32, 64
        rng = np.random.default_rng(17)
        docs = [rng.integers(0, 900, size=int(rng.integers(5, 300))).tolist() for _ in range(400)]
        full = DocIndex(device=d)
        full.initialize(docs, in_memory=True)
        sd, _ = shard_corpus(docs, world, rank, halo)
        ix = DocIndex(device=d)
        ix.initialize(sd, in_memory=True)
        F = [t for doc in reversed(docs) for t in doc]
        starts = np.random.default_rng(5).integers(0, len(F) - 20, size=B)
        pats = [F[a:a + 2] for a in starts]
        dec = ShardedDecoder(ix, V, 10, group=dist.group.WORLD, reduce="peer", halo=halo, peer_barrier="flags")
        ref = ShardedDecoder(full, V, 10)
        dec.start(pats, dev)
        ref.start(pats, dev)
        srng = np.random.default_rng(9)
        bad = []
        for step in range(6):
            tok = [F[a + 2 + step] if srng.random() < 0.85 else int(srng.integers(-1, 900)) for a in starts]
            if step == 3:
                tok = [-1] * B   # every row restarts: every payload row a bitmap
            t = torch.tensor(tok, dtype=torch.int64, device=dev)
            if not torch.equal(dec.step(t), ref.step(t)):
                bad.append(step)
        dec.close()
        ok = not bad
        if bad:
            log(f"peer preflight rank {rank}: masks differ from the unsharded index at steps {bad}")
    except Exception as e:  # reported through the exit status; the parent records it
        log(f"peer preflight rank {rank}: {e!r}")
    finally:
        dist.destroy_process_group()
    return 0 if ok else 1


def peer_preflight(timeout_s: float = PREFLIGHT_TIMEOUT_S, cmd: list | None = None) -> tuple[bool, str]:
    """Run this rank's preflight child (``cmd``: tests substitute a stub) and wait for it, at most
    ``timeout_s`` (then it is killed).  -> (exact, what happened)."""
    import subprocess

    env = dict(os.environ)
    env["FMIDX_PREFLIGHT_PORT"] = str(int(os.environ.get("MASTER_PORT", "29500")) + PREFLIGHT_PORT_OFFSET)
    cmd = cmd or [sys.executable, os.path.abspath(__file__), "--peer-preflight"]
    t0 = time.time()
    try:
        # the child's stdout goes to stderr: stdout carries only the JSON line
        rc = subprocess.run(cmd, env=env, stdout=sys.stderr, stderr=sys.stderr, timeout=timeout_s).returncode
    except subprocess.TimeoutExpired:
        return False, f"timed out after {timeout_s:g} s"
    dt = time.time() - t0
    if rc == 0:
        return True, f"exact ({dt:.1f} s)"
    return False, (f"exit status {rc}" if rc > 0 else f"killed by signal {-rc}") + f" ({dt:.1f} s)"


# ---------------------------------------------------------------------------
WATCHDOG_EXIT = 3   # a leg that hung: the line is printed, the run still fails


class LegWatchdog:
    """A timer that, unless finish() comes first, runs ``on_expiry`` (which prints what
    must still be printed) and ends the process with status ``exit_code`` (default
    WATCHDOG_EXIT = 3: a hang is evidence of a fault, so the launcher and CI see a failed
    run even though the already-measured line is on stdout) -- os._exit, so that a
    thread stuck in a collective or a device wait cannot hold the exit.  finish() and the
    expiry exclude each other: whichever comes second does nothing (a finish() racing the
    expiry waits for the exit)."""

    def __init__(self, seconds: float, on_expiry, exit_code: int = WATCHDOG_EXIT):
        self._lock = threading.Lock()
        self._done = False
        self._on_expiry = on_expiry
        self._code = exit_code
        self._timer = threading.Timer(seconds, self._fire)
        self._timer.daemon = True
        self._timer.start()

    def _fire(self):
        with self._lock:
            if self._done:
                return
            self._done = True
            try:
                self._on_expiry()
            finally:
                sys.stdout.flush()
                sys.stderr.flush()
                os._exit(self._code)

    def finish(self):
        self._timer.cancel()
        with self._lock:
            self._done = True


def main():
    if sys.argv[1:] == ["--peer-preflight"]:
        sys.exit(peer_preflight_child())
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--tokens", type=float, default=float(os.environ.get("FMIDX_BENCH_TOKENS", 4.5e9)))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--corpus", choices=("markov", "paq"), default="markov",
                    help="paq: PAQ-shaped docs (prefix + question + eos, C5) with the paq trace")
    ap.add_argument("--seed", type=int, default=20250905)
    ap.add_argument("--cpu-window", type=int, default=-1,
                    help="CPU baseline: trace steps every leg times (after one untimed warm-up step); "
                         "-1 = enough steps for >= 768 masks per repetition (3 at B = 256, 24 at B = 32)")
    ap.add_argument("--cpu-reps", type=int, default=5, help="CPU baseline: repetitions per leg (median reported)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the gather-ceiling probe")
    ap.add_argument("--no-rank21", action="store_true", help="skip the 2^21-pair rank leg")
    ap.add_argument("--no-sharded", action="store_true", help="N > 1: skip the doc-range sharded leg")
    ap.add_argument("--sharded-at-1", action="store_true",
                    help="run the sharded leg at N = 1 too (one shard; exercises the path on a one-GPU box)")
    ap.add_argument("--sharded-timeout", type=float, default=300.0,
                    help="seconds the doc-range sharded leg may take before the line is printed without it")
    ap.add_argument("--sharded-batches", default="2048",
                    help="global batch sizes the sharded leg runs besides --batch (comma list; '' = none)")
    ap.add_argument("--no-c4", action="store_true",
                    help="N = 1: skip the one-GPU rehearsal of the 8-way doc-range sharded config (C4)")
    ap.add_argument("--packed", action="store_true",
                    help="bit-packed masks (uint32[B, ceil(V/32)]) instead of uint8[B, V] (not the headline)")
    ap.add_argument("--dump-trace", default="", help="write the timed trace states to this .npz")
    ap.add_argument("--eager-replay", action="store_true",
                    help="after the timed region, launch the K timed decode steps and the K standalone LF "
                         "steps once more eagerly (no graph) so PMC counters can be collected per dispatch "
                         "(tools/pmc_traffic.sh)")
    ap.add_argument("--dist-timeout", type=float, default=float(os.environ.get("FMIDX_DIST_TIMEOUT", 600)),
                    help="seconds before a stuck RCCL collective aborts the rank (N > 1)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # plain `python bench.py --gpus N`: this process only launches the ranks and never
        # touches the GPU -- the devices are counted from the KFD topology, not through torch.cuda
        ndev = visible_gpus()
        if ndev < args.gpus:
            print(f"[bench] --gpus {args.gpus} but only {ndev} GPU(s) visible", file=sys.stderr, flush=True)
            sys.exit(2)
        rc = spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])
        sys.exit(rc if rc >= 0 else 128 - rc)
    # the JSON line must be the only thing on stdout, and libraries write there too (RCCL prints its
    # version banner on fd 1 when a communicator comes up): fd 1 now goes to stderr, and the line is
    # written to a duplicate of the original stdout
    line_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    launcher = os.environ.get("FMIDX_BENCH_LAUNCHER", "torchrun" if "WORLD_SIZE" in os.environ else "single")
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE {world} != --gpus {args.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    # one process per GPU: bind the device BEFORE the RCCL communicator exists
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rccl_world = 1
    if world > 1:
        import datetime

        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev, timeout=datetime.timedelta(seconds=args.dist_timeout))
        rccl_world = dist.get_world_size()
        assert rccl_world == args.gpus, f"RCCL world {rccl_world} != --gpus {args.gpus}"
    n_tokens = int(args.tokens)
    B, V, K, W = args.batch, args.vocab, args.steps, max(1, args.warmup)

    fm, text, bwt, build_t = build_index(n_tokens, V, args.seed, dev, args.corpus)
    beg = build_t.pop("beginnings")
    mem_log("index built", dev)
    n = bwt.numel()
    st = fm.stats()
    st["lf_e"] = fm.build_options()["lf_e"] != 0 and n < (1 << 36)
    S = W + K
    if args.cpu_window < 0:
        args.cpu_window = max(3, -(-768 // B))
    cpu_leg = rank == 0 and world == 1 and not args.no_cpu and args.cpu_window > 0 and args.cpu_reps > 0
    # the CPU legs replay steps W .. W + cpu_window of the same trace
    S_trace = max(S, W + args.cpu_window + 1) if cpu_leg else S
    if args.corpus == "paq":
        tokens, init, lo_hist, hi_hist, pats0 = paq_trace(fm, text, bwt, beg, B, V, S_trace, args.seed + rank, dev)
    else:
        tokens, init, lo_hist, hi_hist, pats0 = decode_trace(fm, text, bwt, B, V, S_trace, args.seed + rank, dev)
    # rank throughput at scale: RS_ROWS x (RS_STEPS - 1) independent (state,
    # token) pairs of a wider trace, for one k_lf launch (the grouped kernel)
    rs_tok, rs_lo, rs_hi, rs_ref = rank_pairs(fm, text, bwt, V, args.seed + 17 + rank, dev)
    # ... and 2^21 pairs (4 x the rows), where the library picks the in-wave sweep (query.hip LfTuning)
    r2_tok, r2_lo, r2_hi, r2_ref = (rank_pairs(fm, text, bwt, V, args.seed + 19 + rank, dev, rows=4 * 65536)
                                    if not args.no_rank21 else (None, None, None, None))
    want_sharded = (world > 1 and not args.no_sharded) or args.sharded_at_1
    want_c4 = world == 1 and not args.no_c4 and not args.sharded_at_1 and n > 2e9 and args.corpus == "markov"
    sh = shard_trace(fm, text, bwt, B, V, S, dev) if (want_sharded or want_c4) else None
    # the sharded leg also at the PAQ eval shape's row count (the exchange amortised over more rows)
    shs = None
    if want_sharded:
        shs = {B: sh}
        for b2 in (int(x) for x in args.sharded_batches.split(",") if x.strip()):
            if b2 not in shs:
                shs[b2] = shard_trace(fm, text, bwt, b2, V, S, dev)
    del text
    torch.cuda.empty_cache()
    PK = bool(args.packed)
    mask = (torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev) if PK
            else torch.empty((B, V), dtype=torch.uint8, device=dev))
    lo = init[0].clone()
    hi = init[1].clone()

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
    # the same K steps writing bit-packed rows (uint32 [B, ceil(V/32)]: what the processors'
    # fused epilogue and the sharded exchange consume), reported beside the uint8 headline
    g_packed = None
    if not PK:
        mask_pk = torch.empty((B, (V + 31) // 32), dtype=torch.int32, device=dev)
        bufs_pk = [(torch.empty_like(lo), torch.empty_like(hi)), (torch.empty_like(lo), torch.empty_like(hi))]
        g_packed = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_packed):
            for i in range(K):
                src = (lo, hi) if i == 0 else bufs_pk[i % 2]
                dst = bufs_pk[(i + 1) % 2]
                fm.decode_step(tokens[W + i], src[0], src[1], mask_pk, V, SHIFT, reset_below=0,
                               lo_out=dst[0], hi_out=dst[1], packed=True)

    # Cold runs: the replay has never had its index lines in the caches -- a
    # 1 GiB read-modify-write (4x the 256 MB MALL, far beyond L2) right before
    # it evicts whatever earlier replays (or the trace generation) left there.
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    flush_acc = torch.zeros((), dtype=torch.int64, device=dev)

    def evict(clean=False):
        flush.add_(1)
        if clean:
            # then a 1 GiB read-only pass: the read-modify-write's dirty lines are written back
            # before the timed kernel instead of by its own traffic (profiles/r05_evict/: a 2^19-pair
            # LF launch 78.8 us after the read-modify-write alone, 71.0 after both)
            torch.sum(flush, 0, dtype=torch.int64, out=flush_acc)

    def timed(graph, reps=1, reset=False, cold=False, queued=False):
        # queued (the one-launch rank legs; `graph` is then a callable that launches the
        # kernel directly): the launch is enqueued behind the eviction while the GPU is
        # still busy with it, so the events bracket the kernel itself and not the host's
        # launch latency; a DIRECT launch, not a one-node graph replay, whose own GPU-side
        # cost (~13 us per replay, rocprof kernel trace against the events,
        # profiles/r05_graph_launch/) a 20-step replay spreads over its steps but a
        # one-launch replay would carry whole -- the 1M-request gather ceiling is timed
        # the same way; its eviction is the clean one (evict(clean=True)), since without
        # the host's gap the kernel would otherwise start while the eviction's dirty lines drain
        run = graph.replay if hasattr(graph, "replay") else graph
        ts = []
        if queued:   # one untimed launch: the kernel's first launch in the process loads its code
            run()
            torch.cuda.synchronize()
        for _ in range(reps):
            if reset:
                lo.copy_(state_lo)
                hi.copy_(state_hi)
            if queued:
                torch.cuda.synchronize()
            if cold:
                evict(clean=queued)
            elif queued:
                run()   # warm and queued: the previous launch keeps the GPU busy while this one is enqueued
            if not queued:
                torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            run()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return ts

    # standalone kernels first, then the fused step warm (back-to-back replays
    # of the same trace: its index lines are cache-resident), then the timed
    # region: the fused step cold
    lf_warm = [t / K for t in timed(g_lf, 5)]
    lf_cold = [t / K for t in timed(g_lf, 3, cold=True)]
    # rank throughput at concurrency: all K x B (state, token) pairs of the
    # timed steps in ONE k_lf launch (independent rows), cold
    all_tok = tokens[W:S].reshape(-1).contiguous()
    all_lo = lo_hist[W - 1:S - 1].reshape(-1).contiguous()
    all_hi = hi_hist[W - 1:S - 1].reshape(-1).contiguous()
    big_lo, big_hi = torch.empty_like(all_lo), torch.empty_like(all_hi)
    lfbig_cold = timed(lambda: fm.lf_step_batch(all_tok, all_lo, all_hi, SHIFT, lo_out=big_lo, hi_out=big_hi,
                                                reset_below=0), 5, cold=True, queued=True)
    rs_olo, rs_ohi = torch.empty_like(rs_lo), torch.empty_like(rs_hi)
    rs_cold = timed(lambda: fm.lf_step_batch(rs_tok, rs_lo, rs_hi, SHIFT, lo_out=rs_olo, hi_out=rs_ohi,
                                             reset_below=0), 5, cold=True, queued=True)
    log(f"rank 2^19 cold launches (us, median reported): {', '.join(f'{t * 1e3:.1f}' for t in rs_cold)}")
    rs_ok = bool(torch.equal(rs_olo, rs_ref[0]) and torch.equal(rs_ohi, rs_ref[1]))
    r2 = None
    if r2_tok is not None:
        r2_olo, r2_ohi = torch.empty_like(r2_lo), torch.empty_like(r2_hi)

        def r2_launch():
            fm.lf_step_batch(r2_tok, r2_lo, r2_hi, SHIFT, lo_out=r2_olo, hi_out=r2_ohi, reset_below=0)
        r2_cold = timed(r2_launch, 5, cold=True, queued=True)
        r2_warm = timed(r2_launch, 3, queued=True)
        r2 = {"rows": int(r2_tok.numel()), "avg_launch_us_cold": float(np.median(r2_cold)) * 1e3,
              "avg_launch_us_warm": float(np.median(r2_warm)) * 1e3,
              "matches_decode_kernel": bool(torch.equal(r2_olo, r2_ref[0]) and torch.equal(r2_ohi, r2_ref[1]))}
        del r2_olo, r2_ohi
    mask_ms = [t / K for t in timed(g_mask, 5)]
    packed_cold = None
    if g_packed is not None:
        packed_warm = [t / K for t in timed(g_packed, 3, reset=True)]
        packed_cold = [t / K for t in timed(g_packed, 3, reset=True, cold=True)]
    step_warm = [t / K for t in timed(g_step, 3, reset=True)]
    lo.copy_(state_lo)
    hi.copy_(state_hi)
    evict()
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
        for i in range(K):
            fm.lf_step_batch(tokens[W + i], lo_hist[W + i - 1], hi_hist[W + i - 1], SHIFT,
                             lo_out=lo_scr, hi_out=hi_scr, reset_below=0)
        torch.cuda.synchronize()
    del flush
    if args.dump_trace and rank == 0:
        np.savez_compressed(args.dump_trace, tokens=tokens[:S].cpu().numpy(), lo=lo_hist[:S].cpu().numpy(),
                            hi=hi_hist[:S].cpu().numpy(), n=n, warmup=W)
    # ---- roofline accounting for the dominant (fused decode) kernel
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
    pcached = fm.cache_contains(lo_hist[W - 1:S - 1].reshape(-1).contiguous(),
                                hi_hist[W - 1:S - 1].reshape(-1).contiguous()).view(K, B).cpu().numpy()
    read_bytes = np.stack([plan_bytes(lo_np[i], hi_np[i], n, b0_log2, bm_levels, words * 4, follow[i], cached[i])
                           for i in range(K)])
    mask_bytes_per_launch = float((read_bytes.sum(1) + (B * ((V + 31) // 32) * 4 if PK else B * V)).mean())
    mask_us = float(np.median(mask_ms)) * 1e3
    # LF bytes per launch, by the plan each kernel executes (lf_plan_bytes)
    lf_dec = np.stack([lf_plan_bytes(prev_lo[i], prev_hi[i], tok_np[i], n, pcached[i], st, "decode")
                       for i in range(K)]).sum(1)
    lf_std = np.stack([lf_plan_bytes(prev_lo[i], prev_hi[i], tok_np[i], n, pcached[i], st, "lf")
                       for i in range(K)]).sum(1)
    lf_us_warm = float(np.median(lf_warm)) * 1e3
    lf_us_cold = float(np.median(lf_cold)) * 1e3
    rank_gbs = float(lf_std.mean()) / (lf_us_cold * 1e-6) / 1e9
    lfbig_us = float(np.median(lfbig_cold)) * 1e3
    rank_gbs_big = float(lf_std.sum()) / (lfbig_us * 1e-6) / 1e9
    rs_pc = fm.cache_contains(rs_lo, rs_hi).cpu().numpy()
    rs_bytes = float(lf_plan_bytes(rs_lo.cpu().numpy(), rs_hi.cpu().numpy(), rs_tok.cpu().numpy(), n, rs_pc, st,
                                   "lf").sum())
    rs_us = float(np.median(rs_cold)) * 1e3
    rank_gbs_scale = rs_bytes / (rs_us * 1e-6) / 1e9
    if r2 is not None:
        r2_pc = fm.cache_contains(r2_lo, r2_hi).cpu().numpy()
        r2["alg_bytes_per_launch"] = float(lf_plan_bytes(r2_lo.cpu().numpy(), r2_hi.cpu().numpy(),
                                                         r2_tok.cpu().numpy(), n, r2_pc, st, "lf").sum())
        r2["rank_GBps"] = r2["alg_bytes_per_launch"] / (r2["avg_launch_us_cold"] * 1e-6) / 1e9
        r2["frac_of_peak"] = r2["rank_GBps"] / HBM_PEAK_GBS
        r2["lf_steps_per_s"] = r2["rows"] / (r2["avg_launch_us_cold"] * 1e-6)
        r2["kernel"] = "k_lf_sweep<true> (in-wave tail rows), chosen by the library from 2^18 rows"
        log(f"rank at 2^21 pairs: {r2['avg_launch_us_cold']:.1f}us cold ({r2['avg_launch_us_warm']:.1f} warm), "
            f"{r2['rank_GBps']:.0f} GB/s, {r2['lf_steps_per_s'] / 1e9:.1f} G steps/s, exact {r2['matches_decode_kernel']}")
    gather_gbs, chase_ns, gather_modes = (None, None, None)
    if not args.no_gather:
        gather_gbs, chase_ns, gather_modes = gather_ceiling(dev)
        log(f"gather ceiling: {gather_gbs:.0f} GB/s best independent random 64-B lines "
            f"({', '.join(f'{k} {v:.0f}' for k, v in gather_modes.items())}); "
            f"dependent chase {chase_ns:.0f} ns/hop (256 chains)")
    # dominant kernel = the fused k_decode (one launch per step)
    decode_bytes = mask_bytes_per_launch + float(lf_dec.mean())
    decode_us = step_ms * 1e3
    achieved = decode_bytes / (decode_us * 1e-6) / 1e9
    widths = (hi_np - lo_np)
    log(f"step cold {step_ms * 1e3:.1f}us, warm [{', '.join(f'{t * 1e3:.1f}' for t in step_warm)}] "
        f"(standalone lf cold {lf_us_cold:.1f}us / warm {lf_us_warm:.1f}us, {K * B} rows in one launch "
        f"{lfbig_us:.1f}us = {rank_gbs_big:.0f} GB/s, {rs_tok.numel()} rows {rs_us:.1f}us = {rank_gbs_scale:.0f} GB/s "
        f"(exact {rs_ok}), mask {mask_us:.1f}us, "
        f"wall/step {wall / K * 1e6:.1f}us, graph) bytes/step {decode_bytes / 1e6:.2f}MB -> {achieved:.0f} GB/s; "
        f"live rows {(widths > 0).mean():.2f}, median width {np.median(widths[widths > 0]) if (widths > 0).any() else 0}, "
        f"cached rows {cached.mean():.3f} (cache: {st['cache_nodes']} ranges >= {st['cache_min']}, "
        f"{st['cache_bytes'] / 2**30:.1f} GiB; transitions {st['trans_entries']} "
        f"(+{st['trans_dropped']} left out), {st['trans_bytes'] / 2**30:.1f} GiB)")

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "masks/s",
        "n_gpus": world,
        "rccl_world": rccl_world,
        "launcher": launcher,
        "steps": K,
        "warmup": W,
        "ms_per_step": step_ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "uint64",
        "data": "synthetic",
        "config": {
            "workload": (f"decode step (LF + allowed-token mask) over a synthetic PAQ-shaped corpus (~24-token docs, "
                         f"shared 3-token prefix + question + eos) of n={n} tokens (C5), B={B} rows whose patterns "
                         f"start from the prefix (force_decoding_from), V={V}, incremental ranges; timed replay "
                         f"cold (caches evicted)" if args.corpus == "paq" else
                         f"decode step (LF + allowed-token mask) over a synthetic Markov/Zipf corpus "
                         f"of n={n} tokens ({'C3 enwiki scale' if n > 2e9 else ('C2 simplewiki scale' if n <= 3.5e8 else 'Markov corpus between the C2 and C3 scales; C5 is --corpus paq')}"
                         f"), B={B} rows, V={V}, incremental ranges; timed replay cold (caches evicted)"),
            "corpus": args.corpus,
            "corpus_tokens": n,
            "global_batch": world * B,
            "batch_per_gpu": B,
            "vocab": V,
            "wavelet_digit_levels": st["levels"],
            "parallelism": f"replicas{world}",
            "mask": "uint32[B,ceil(V/32)] bit-packed" if PK else "uint8[B,V]",
        },
        "cold_ms_per_step": step_ms,
        "packed_output": None if packed_cold is None else {
            "mask": "uint32[B,ceil(V/32)] bit-packed (the layout the processors' fused epilogue and the sharded "
                    "exchange read)",
            "cold_ms_per_step": float(np.median(packed_cold)), "warm_ms_per_step": float(np.median(packed_warm)),
            "value_cold": B / (float(np.median(packed_cold)) * 1e-3)},
        "warm_ms_per_step": float(np.median(step_warm)),
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
            "timing": "cold: the timed replay follows a 1 GiB cache eviction",
            # also against the measured stream rate of MI355X_MICROARCH.md
            "peak_stream_measured": HBM_STREAM_GBS,
            "frac_stream": achieved / HBM_STREAM_GBS,
        },
        "standalone_kernels": {
            "k_lf": {"avg_launch_us_cold": lf_us_cold, "avg_launch_us_warm": lf_us_warm,
                     "alg_bytes_per_launch": float(lf_std.mean()), "rank_GBps": rank_gbs,
                     "rank_frac_of_peak": rank_gbs / HBM_PEAK_GBS,
                     "gather_ceiling_GBps": gather_gbs,
                     "rank_frac_of_gather_ceiling": (rank_gbs / gather_gbs) if gather_gbs else None,
                     "dependent_hop_ns": chase_ns,
                     "batched": {"rows": int(K * B), "avg_launch_us_cold": lfbig_us,
                                 "alg_bytes_per_launch": float(lf_std.sum()), "rank_GBps": rank_gbs_big,
                                 "rank_frac_of_gather_ceiling": (rank_gbs_big / gather_gbs) if gather_gbs else None,
                                 "note": "all K x B (state, token) pairs of the timed steps in one launch"},
                     "at_scale": {"rows": int(rs_tok.numel()), "avg_launch_us_cold": rs_us,
                                  "cold_launches_us": [t * 1e3 for t in rs_cold],
                                  "alg_bytes_per_launch": rs_bytes, "rank_GBps": rank_gbs_scale,
                                  "rank_frac_of_peak": rank_gbs_scale / HBM_PEAK_GBS,
                                  "rank_frac_of_gather_ceiling": (rank_gbs_scale / gather_gbs) if gather_gbs else None,
                                  "M_lf_steps_per_s": rs_tok.numel() / (rs_us * 1e-6) / 1e6,
                                  "matches_decode_kernel": rs_ok,
                                  "note": "2^19 independent (state, token) pairs of a 65536-row trace in one k_lf launch "
                                          "(the in-wave sweep k_lf_sweep<true>, which the library picks from 2^18 rows: one lane per row, narrow rows packed, cached rows probed eight per round trip, tail rows in-wave), cold after a clean eviction, one direct launch timed queued behind it (no graph node)"},
                     "bytes_model": "64-B lines the LF plan reads per live row (bench.lf_plan_bytes)"},
            "k_decode_mask_only": {"avg_launch_us": mask_us, "alg_bytes_per_launch": mask_bytes_per_launch,
                                   "GBps": mask_bytes_per_launch / (mask_us * 1e-6) / 1e9},
        },
        "device_bytes": st["device_bytes"],
        # the BWT copy the bench materialised for its trace and the CPU baseline (fm_device_bwt):
        # held by the handle beside the query structures, not one of them
        "bwt_view_bytes": st.get("bwt_view_bytes", 0),
        "held_device_bytes": st["device_bytes"] + st.get("bwt_view_bytes", 0),
        "index": {"build": build_t, **st},
        "trace_check": ok,
        # the metric's second half ("rank GB/s vs HBM roofline"), summarised: LF throughput at
        # concurrency (2^19 independent steps, one grouped launch, cold) against 8 TB/s and the live
        # random-64-B gather ceiling; at B = 256 the LF launch is a latency chain (k_lf above)
        "rank": {"GBps": rank_gbs_scale, "unit": "GB/s", "peak": HBM_PEAK_GBS,
                 "frac_of_peak": rank_gbs_scale / HBM_PEAK_GBS,
                 "gather_ceiling_GBps": gather_gbs,
                 "gather_ceiling_by_shape_GBps": gather_modes,
                 "frac_of_gather_ceiling": (rank_gbs_scale / gather_gbs) if gather_gbs else None,
                 "lf_steps_per_s": rs_tok.numel() / (rs_us * 1e-6),
                 "b256_GBps": rank_gbs, "b256_avg_launch_us_cold": lf_us_cold,
                 "pairs_2_21": r2,
                 "timing": "each launch direct (not a one-node graph replay: ~13 us of GPU-side cost per replay, "
                           "profiles/r05_graph_launch/), enqueued behind a clean 1 GiB eviction, median of 5, as "
                           "the 1M-request gather ceiling"},
    }
    # PMC traffic (tools/pmc_traffic.sh) is collected in a separate rocprofv3 run and committed;
    # it is used only when it was counted on this very library build, config and mask layout
    # one committed file per config: profiles/pmc_traffic.json (C3), pmc_traffic_c2.json, pmc_traffic_c5.json
    import glob

    lib_hash = lib_sha16()
    result["roofline"]["lib_sha16"] = lib_hash
    seen = []
    for pmc in sorted(glob.glob(os.path.join(REPO, "profiles", "pmc_traffic*.json"))):
        try:
            with open(pmc) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        name = os.path.relpath(pmc, REPO)
        seen.append(f"{name}: lib {t.get('lib_sha16')} n={t.get('corpus_tokens')} B={t.get('batch')}")
        if t.get("lib_sha16") == lib_hash and t.get("corpus_tokens") == n and t.get("batch") == B and not PK:
            result["roofline"]["traffic"] = t.get("k_decode_bytes_per_launch")
            result["roofline"]["traffic_source"] = f"{name} (same lib_sha16, n, B)"
            if t.get("k_lf_bytes_per_launch") is not None:
                result["standalone_kernels"]["k_lf"]["pmc_bytes_per_launch"] = t["k_lf_bytes_per_launch"]
            break
    else:
        result["roofline"]["traffic_source"] = (f"none counted for this run (lib {lib_hash}, n={n}, B={B}); "
                                                f"committed: {'; '.join(seen) or 'none'}")
    pr = os.path.join(REPO, "profiles", "pmc_rank.json")
    if os.path.exists(pr) and n > 4e9:
        try:   # tools/pmc_rank.sh: the 2^19-row grouped launches of tools/probe_rank.py on a C3 index
            with open(pr) as f:
                t = json.load(f)
            big = [(a, b) for a, b in zip(t["fetch_bytes"], t["write_bytes"]) if b >= 8e6]
            if t.get("lib_sha16") != lib_hash:
                big = []
            if big:
                at = result["standalone_kernels"]["k_lf"]["at_scale"]
                at["pmc_bytes_per_launch"] = float(np.median([a + b for a, b in big]))
                if at.get("alg_bytes_per_launch"):   # HBM bytes moved per byte of LF plan
                    at["pmc_over_plan_bytes"] = at["pmc_bytes_per_launch"] / at["alg_bytes_per_launch"]
        except Exception:
            pass
    # Memory-side read requests by size (tools/pmc_req.sh, committed under profiles/ with the
    # library hash): on gfx950 every random read -- 8 B, a 64-B line, a 128-B line -- is one
    # 128-B request (tools/pmc_gather_calib.py), so the random-read ceiling is a REQUEST rate,
    # measured live here by the gather shapes (one request per line for the cooperative shapes
    # and the 8-B words), and a kernel's requests per launch say what it really moved.
    gm = gather_modes or {}
    req_ceiling = max(gm.get("coop8_128B", 0) / 128, gm.get("coop4_64B", 0) / 64,
                      gm.get("lane_8B", 0) / 8)          # G requests/s (GB/s / B per request)
    result["rank"]["request_ceiling_G_per_s"] = req_ceiling
    # the same at the launch's own size, cold (gather_ceiling: ~1M requests after an eviction)
    req_ceiling_1m = max(gm.get("coop8_128B_1M_cold", 0) / 128, gm.get("lane_8B_1M_cold", 0) / 8)
    result["rank"]["request_ceiling_1M_cold_G_per_s"] = req_ceiling_1m
    # the rank figure comes from this bench's own 2^19-pair launch (pmc_req_c3.json, counted over the
    # same command) when that file has it, else from tools/probe_rank.py's launch of the same shape
    have_c3_rank = False

    def rank_2_19(r):
        # a 2^19-row LF launch (grouped kernel or in-wave sweep): 8.4 MB of new states written
        # (the 2^21 launch writes 33.5 MB, the by-path launches less)
        return ("k_lf_group" in r["kernel"] or "k_lf_sweep" in r["kernel"]) and 8e6 <= r.get("write_bytes", 0) < 2e7

    try:
        with open(os.path.join(REPO, "profiles", "pmc_req_c3.json")) as f:
            have_c3_rank = any(rank_2_19(r) for r in json.load(f)["dispatches"])
    except (OSError, ValueError, KeyError):
        pass
    for name, where in ((("pmc_req_c3.json" if have_c3_rank else "pmc_req_rank.json"), "rank"),
                        ("pmc_req_c3.json", "roofline")):
        path = os.path.join(REPO, "profiles", name)
        if not os.path.exists(path) or n < 4e9:
            continue
        try:
            with open(path) as f:
                t = json.load(f)
            if t.get("lib_sha16") != lib_hash:
                result[where]["pmc_requests_source"] = f"none: profiles/{name} was counted on lib {t.get('lib_sha16')}"
                continue
            if where == "rank":      # the 2^19-row launches (the by-path launches write less)
                rows = [r for r in t["dispatches"] if rank_2_19(r)]
            else:                    # the uint8 decode launches of the C3 bench (B = 256)
                rows = [r for r in t["dispatches"] if "k_decode<false, true" in r["kernel"]]
            if not rows:
                continue
            req = float(np.median([r["rdreq"] for r in rows]))
            rd = float(np.median([r["read_bytes"] for r in rows]))
            wr = float(np.median([r["write_bytes"] for r in rows]))
            us = rs_us if where == "rank" else decode_us
            result[where].update({
                "pmc_requests_per_launch": req, "pmc_read_bytes_per_launch": rd, "pmc_write_bytes_per_launch": wr,
                "pmc_hbm_GBps": (rd + wr) / (us * 1e-6) / 1e9,
                "pmc_requests_source": f"profiles/{name} (same lib_sha16; {len(rows)} launches, median)"})
            if where == "rank":
                rate = req / (us * 1e-6) / 1e9
                result["rank"]["request_rate_G_per_s"] = rate
                result["rank"]["frac_of_request_ceiling"] = rate / req_ceiling if req_ceiling else None
                result["rank"]["frac_of_request_ceiling_1M_cold"] = rate / req_ceiling_1m if req_ceiling_1m else None
                # the 2^21-pair launches of the same file (33.5 MB of new states written each)
                r21 = [r for r in t["dispatches"] if "k_lf_sweep" in r["kernel"] and 3e7 <= r.get("write_bytes", 0) < 4e7]
                p21 = result["rank"].get("pairs_2_21")
                if r21 and p21 and p21.get("avg_launch_us_cold"):
                    req21 = float(np.median([r["rdreq"] for r in r21]))
                    rate21 = req21 / (p21["avg_launch_us_cold"] * 1e-6) / 1e9
                    p21.update({"pmc_requests_per_launch": req21, "request_rate_G_per_s": rate21,
                                "frac_of_request_ceiling": rate21 / req_ceiling if req_ceiling else None,
                                "frac_of_request_ceiling_1M_cold": rate21 / req_ceiling_1m if req_ceiling_1m else None})
        except Exception as e:
            result[where]["pmc_requests_source"] = f"unreadable: {e!r}"
    if cpu_leg:
        try:
            result["cpu_baseline"] = cpu_baseline(fm, bwt, tokens, lo_hist, hi_hist, pats0, V, W,
                                                  args.cpu_window, args.cpu_reps, dev)
        except Exception as e:  # the GPU line must still print
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if want_sharded and world > 1 and os.environ.get("FMIDX_BENCH_PEER", "1") != "0":
        # the peer modes' cross-device mechanics, first in a child process (see peer_preflight)
        import torch.distributed as dist

        pf_ok, pf_note = peer_preflight()
        log(f"peer preflight: {pf_note}")
        agree = torch.tensor([1 if pf_ok else 0], device=dev)
        dist.all_reduce(agree, op=dist.ReduceOp.MIN)
        result["peer_preflight"] = {"exact_every_rank": bool(agree.item()), "rank0": pf_note}
        if not int(agree.item()):
            os.environ["FMIDX_BENCH_PEER"] = "0"   # the sharded leg's dense and sparse modes still run
    if want_sharded:
        if world == 1:
            import torch.distributed as dist

            if not dist.is_initialized():
                dist.init_process_group("nccl", device_id=dev, init_method="tcp://127.0.0.1:29533",
                                        world_size=1, rank=0)
        holder = [bwt, fm]
        del bwt, fm
        torch.cuda.empty_cache()
        # Watchdog: the replica line is already measured; a sharded leg stuck in a collective or a
        # peer wait (first run over more than one rank on a new node) must not take it down.  Every
        # rank arms its own timer; on expiry rank 0 prints the line with the leg marked as timed out
        # and every rank leaves with status WATCHDOG_EXIT (3: the run fails, the measured line is still
        # on stdout; os._exit: no teardown of the stuck communicator).
        def on_stuck():
            result["sharded"] = {"value": None,
                                 "error": f"watchdog: the sharded leg did not finish within {args.sharded_timeout:g} s"}
            log(result["sharded"]["error"])
            if rank == 0:
                line_out.write(json.dumps(result) + "\n")
                line_out.flush()

        dog = LegWatchdog(args.sharded_timeout, on_stuck)
        try:
            result["sharded"] = sharded_leg(holder, args.seed, n_tokens, V, K, W, world, rank, dev, shs)
            log(f"sharded: {result['sharded']['value'] / 1e6:.2f} M masks/s, "
                f"{result['sharded']['ms_per_step'] * 1e3:.1f} us/step, exact {result['sharded']['masks_equal_unsharded']}")
        except Exception as e:  # the replica line must still print
            result["sharded"] = {"value": None, "error": repr(e)}
        dog.finish()
    elif want_c4:
        holder = [bwt, fm]
        del bwt, fm
        gc.collect()
        torch.cuda.empty_cache()
        mem_log("before the after-replica legs (replica still held)", dev)
        try:
            main_trace = (tokens[W:S], state_lo, state_hi, lo_hist[S - 1], hi_hist[S - 1])
            result["compact_profile"], result["c4_one_gpu"] = after_replica_legs(
                holder, args.seed, n_tokens, V, B, K, W, dev, main_trace, sh)
            c4 = result["c4_one_gpu"]
            if "error" in c4:
                log(f"c4 on one GPU failed: {c4['error']}")
            else:
                log(f"c4 on one GPU: slowest shard {c4['slowest_shard_cold_us']:.1f}us cold, OR "
                    f"{c4['or_pass_cold_us']:.1f}us, exact {c4['masks_equal_unsharded']}, predicted 8-GPU step "
                    f"{c4['predicted_step_us']['direct']:.0f}-{c4['predicted_step_us']['ring']:.0f}us (dense), "
                    f"{c4['peer_exchange']['predicted_step_us']:.0f}us (peer; "
                    f"{c4['peer_exchange']['predicted_step_us_flags']:.0f}us with the flag barrier; OR pass "
                    f"{c4['peer_exchange']['or_rows_peers_cold_us']:.1f}us, exact "
                    f"{c4['peer_exchange']['masks_equal_unsharded']})")
        except Exception as e:  # the replica line must still print
            result["c4_one_gpu"] = {"error": repr(e)}
    if rank == 0:
        line_out.write(json.dumps(result) + "\n")
        line_out.flush()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
