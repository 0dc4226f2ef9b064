"""Rank (LF-step) throughput at concurrency vs the random-gather ceiling
(the "rank GB/s vs HBM roofline" half of BASELINE's metric).

At B = 256 one LF launch is a latency chain (a few dependent round trips per
row), so its GB/s says nothing about how well the rank kernel uses HBM.  Here
the same k_lf kernel (fm_lf_step_batch) runs over R = 2^13 .. 2^19 independent
(state, token) pairs of a decode trace on the C3-scale index, in ONE launch,
cold (1 GiB eviction first) and warm; bytes = bench.lf_plan_bytes (the 64-B
lines each row's LF plan reads).  The ceiling is k_gather64 (independent
random 64-B lines) over an 8 GiB buffer and over the index's own 16.8 GiB BWT
allocation (TLB reach at index scale).  Also: get_range (k_search) over many
true patterns, as LF steps per second.

usage: python tools/probe_rank.py [--tokens 4.5e9] [--rows-log2 13,15,17,19]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "fm-index-constrained-decoding_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from fmidx._lib import check, lib  # noqa: E402
from fmidx.synth import decode_trace  # noqa: E402

SHIFT = bench.SHIFT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=float, default=4.5e9)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--rows-log2", default="13,15,17,19")
    ap.add_argument("--steps", type=int, default=9, help="trace steps (pairs = rows x (steps - 1))")
    ap.add_argument("--patterns", type=int, default=1 << 18)
    ap.add_argument("--out", default="")
    ap.add_argument("--by-path", action="store_true", help="also one launch per LF path class (PMC breakdown)")
    ap.add_argument("--sorted", action="store_true",
                    help="also each launch with its pairs ordered by lo (locality experiment, sort untimed)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    fm, text, bwt, _ = bench.build_index(int(args.tokens), args.vocab, 20250905, dev)
    n = bwt.numel()
    st = fm.stats()
    st["lf_e"] = fm.build_options()["lf_e"] != 0
    stream = torch.cuda.current_stream(dev).cuda_stream
    sink = torch.zeros(1024, dtype=torch.int64, device=dev)
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)
    res = {"corpus_tokens": n, "vocab": args.vocab}

    def timed(fn, cold, reps=3):
        best = None
        for _ in range(reps):
            if cold:
                flush.add_(1)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        return best

    # ---- gather ceilings
    def gather(ptr, nbytes, cold, mode=0):
        threads, loads = 256 * 4096, 64
        _, lpl, line = bench.GATHER_MODES[mode]
        ms = timed(lambda: check(lib().fm_probe_gather(ptr, nbytes, mode, loads, threads, sink.data_ptr(), stream),
                                 "probe"), cold)
        return threads // lpl * loads * line / (ms * 1e-3) / 1e9

    buf = torch.randint(0, 1 << 62, (1 << 30,), dtype=torch.int64, device=dev)
    res["gather_8GiB_GBps"] = gather(buf.data_ptr(), 8 << 30, True)
    res["gather_8GiB_by_shape_GBps"] = {bench.GATHER_MODES[m][0]: gather(buf.data_ptr(), 8 << 30, True, m)
                                        for m in bench.GATHER_MODES}
    del buf
    torch.cuda.empty_cache()
    res["gather_bwt_by_shape_GBps"] = {bench.GATHER_MODES[m][0]: gather(bwt.data_ptr(), bwt.numel() * 4, True, m)
                                       for m in bench.GATHER_MODES}
    res["gather_bwt_GBps"] = max(res["gather_bwt_by_shape_GBps"]["lane_64B"],
                                 res["gather_bwt_by_shape_GBps"]["coop4_64B"])
    print(f"gather ceiling: 8 GiB {res['gather_8GiB_GBps']:.0f} GB/s, index BWT "
          f"({bwt.numel() * 4 / 2**30:.1f} GiB) {res['gather_bwt_GBps']:.0f} GB/s", flush=True)

    # ---- k_lf over R x (S - 1) independent pairs, one launch
    res["k_lf"] = []
    for rl in [int(x) for x in args.rows_log2.split(",") if x]:
        R = 1 << rl
        S = args.steps
        rows_per = max(1, R // (S - 1))
        tokens, _, lo_h, hi_h, _ = decode_trace(fm, text, bwt, rows_per, args.vocab, S, 4242 + rl, dev)
        tok = tokens[1:S].reshape(-1).contiguous()
        plo = lo_h[0:S - 1].reshape(-1).contiguous()
        phi = hi_h[0:S - 1].reshape(-1).contiguous()
        m = tok.numel()
        olo, ohi = torch.empty_like(plo), torch.empty_like(phi)
        pc = fm.cache_contains(plo, phi).cpu().numpy()
        by = bench.lf_plan_bytes(plo.cpu().numpy(), phi.cpu().numpy(), tok.cpu().numpy(), n, pc, st, "lf")
        fn = lambda: fm.lf_step_batch(tok, plo, phi, SHIFT, lo_out=olo, hi_out=ohi, reset_below=0)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        ok = bool(torch.equal(olo, lo_h[1:S].reshape(-1)) and torch.equal(ohi, hi_h[1:S].reshape(-1)))
        cold = timed(fn, True)
        warm = timed(fn, False)
        w = (phi - plo).cpu().numpy()
        live = (tok.cpu().numpy() >= 0) & (w > 0)
        e = {"rows": m, "cold_us": cold * 1e3, "warm_us": warm * 1e3, "bytes": int(by.sum()),
             "GBps_cold": by.sum() / (cold * 1e-3) / 1e9, "GBps_warm": by.sum() / (warm * 1e-3) / 1e9,
             "Msteps_per_s_cold": m / (cold * 1e-3) / 1e6, "matches_trace": ok,
             "live": float(live.mean()), "cached_parent": float(pc.mean()),
             "narrow_le512": float((live & (w <= 512)).mean())}
        e["frac_gather_bwt_cold"] = e["GBps_cold"] / res["gather_bwt_GBps"]
        res["k_lf"].append(e)
        print(f"k_lf rows {m:7d}: cold {cold * 1e3:8.1f} us ({e['GBps_cold']:6.0f} GB/s, "
              f"{e['Msteps_per_s_cold']:7.0f} M steps/s, {e['frac_gather_bwt_cold']:.3f} of gather), warm "
              f"{warm * 1e3:8.1f} us ({e['GBps_warm']:6.0f} GB/s); {by.sum() / m:.0f} B/row, exact {ok}",
              flush=True)
        if args.sorted:
            order = torch.argsort(plo)
            st_, sl_, sh_ = tok[order].contiguous(), plo[order].contiguous(), phi[order].contiguous()
            fs = lambda: fm.lf_step_batch(st_, sl_, sh_, SHIFT, lo_out=olo, hi_out=ohi, reset_below=0)  # noqa: E731
            fs()
            torch.cuda.synchronize()
            e["sorted_exact"] = bool(torch.equal(olo, lo_h[1:S].reshape(-1)[order]) and
                                     torch.equal(ohi, hi_h[1:S].reshape(-1)[order]))
            e["sorted_cold_us"] = timed(fs, True) * 1e3
            e["sorted_warm_us"] = timed(fs, False) * 1e3
            print(f"   sorted by lo: cold {e['sorted_cold_us']:.1f} us, warm {e['sorted_warm_us']:.1f} us, "
                  f"exact {e['sorted_exact']}", flush=True)
        del tokens, lo_h, hi_h, tok, plo, phi, olo, ohi
        torch.cuda.empty_cache()

    # ---- the last (largest) launch split by LF path: one grouped launch per class
    # (tuning lf_group_min = 0 through fm_set_tuning, so even a small class takes the
    # grouped kernel), each cold, bytes by the LF plan.  With tools/pmc_rank.sh the
    # LAST len(by_path) k_lf_group dispatches are these, in this order.
    if args.by_path:
        from fmidx.options import set_tuning

        old_tuning = set_tuning(lf_group_min=0)
        R = 1 << max(int(x) for x in args.rows_log2.split(",") if x)
        S = args.steps
        tokens, _, lo_h, hi_h, _ = decode_trace(fm, text, bwt, max(1, R // (S - 1)), args.vocab, S, 777, dev)
        tok = tokens[1:S].reshape(-1).contiguous()
        plo = lo_h[0:S - 1].reshape(-1).contiguous()
        phi = hi_h[0:S - 1].reshape(-1).contiguous()
        pc = fm.cache_contains(plo, phi).cpu().numpy().astype(bool)
        t_np, l_np, h_np = tok.cpu().numpy(), plo.cpu().numpy(), np.minimum(phi.cpu().numpy(), n)
        w = h_np - l_np
        live = (t_np >= 0) & (w > 0)
        full = live & (l_np == 0) & (h_np == n)
        cmin = st["cache_min"] or (1 << 62)
        cls = {"full_range": full,
               "group_e_scan_le16": live & ~full & (w <= 16),
               "quad_e_scan_17_128": live & ~full & (w > 16) & (w <= 128),
               "probe_cached_parent": live & ~full & (w >= cmin) & pc,
               "wave_e_scan_129_512": live & ~full & (w > 128) & (w <= 512),
               "descent_or_other": live & ~full & (w > 512) & ~((w >= cmin) & pc),
               "dead_or_restart": ~live}
        res["by_path"] = []
        for name, sel in cls.items():
            idx = torch.tensor(np.flatnonzero(sel), dtype=torch.int64, device=dev)
            if idx.numel() == 0:
                continue
            t_, l_, h_ = tok[idx].contiguous(), plo[idx].contiguous(), phi[idx].contiguous()
            ol, oh = torch.empty_like(l_), torch.empty_like(h_)
            by = bench.lf_plan_bytes(l_.cpu().numpy(), h_.cpu().numpy(), t_.cpu().numpy(), n, pc[sel], st, "lf")
            flush.add_(1)
            torch.cuda.synchronize()
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            fm.lf_step_batch(t_, l_, h_, SHIFT, lo_out=ol, hi_out=oh, reset_below=0)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3
            ok = bool(torch.equal(ol, lo_h[1:S].reshape(-1)[idx]) and torch.equal(oh, hi_h[1:S].reshape(-1)[idx]))
            e = {"path": name, "rows": int(idx.numel()), "alg_bytes": int(by.sum()), "cold_us": us,
                 "GBps": by.sum() / (us * 1e-6) / 1e9, "exact": ok}
            res["by_path"].append(e)
            print(f"by path {name:22s} {e['rows']:7d} rows {us:8.1f} us {e['GBps']:7.0f} GB/s "
                  f"({by.sum() / max(1, e['rows']):.0f} B/row), exact {ok}", flush=True)
        set_tuning(old_tuning)

    # ---- get_range (k_search) over P true patterns of U{1..32} tokens
    P = args.patterns
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    lens = torch.randint(1, 33, (P,), generator=g, device=dev)
    q = torch.randint(0, n - 40, (P,), generator=g, device=dev)
    offs = torch.zeros(P + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=offs[1:])
    tot = int(offs[-1].item())
    row_of = torch.repeat_interleave(torch.arange(P, device=dev), lens)
    k = torch.arange(tot, device=dev) - offs[:-1][row_of]
    toks = text[(n - 2) - (q[row_of] + k)].to(torch.int64) - SHIFT
    lo = torch.zeros(P, dtype=torch.int64, device=dev)
    hi = torch.zeros(P, dtype=torch.int64, device=dev)
    fn = lambda: fm.backward_search_batch(toks, offs, SHIFT, lo, hi)  # noqa: E731
    cold = timed(fn, True)
    warm = timed(fn, False)
    nonempty = float((hi > lo).float().mean().item())
    res["k_search"] = {"patterns": P, "tokens": tot, "cold_us": cold * 1e3, "warm_us": warm * 1e3,
                       "Msteps_per_s_cold": tot / (cold * 1e-3) / 1e6, "nonempty": nonempty}
    print(f"get_range {P} patterns / {tot} tokens: cold {cold * 1e3:.0f} us = "
          f"{res['k_search']['Msteps_per_s_cold']:.0f} M LF steps/s (warm {warm * 1e3:.0f} us), "
          f"non-empty {nonempty:.3f}", flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"[probe_rank] {time.time() - t0:.0f}s", file=sys.stderr)
