#!/usr/bin/env python
"""The sparse exchange's OR pass (fm_shard_or_rows) against the dense one
(fm_or_bits) on synthetic payloads of the C4 shape: P = 8 parts, B = 256
rows, V = 128256; per part and row a dense bitmap with probability
--dense (density 10 %) else a list of ~Geometric(--mean) random symbols.
Both are timed as the bench times its OR pass: K launches in one graph, each
over its own copy of the gathered data, after a 1 GiB eviction (cold) and
back to back (warm).  The outputs must agree.

    python tools/bench_or_rows.py [--wide 0.15]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fm-index-constrained-decoding_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--dense", type=float, default=0.15)
    ap.add_argument("--mean", type=float, default=6.0)
    ap.add_argument("--wide", type=float, default=0.0, help="fraction of rows dense on EVERY part (wide rows)")
    ap.add_argument("-K", type=int, default=20)
    args = ap.parse_args()
    from fmidx.sharding import or_bits, or_payloads

    P, B, V, SH = args.parts, args.rows, args.vocab, 10
    W = (V + 31) // 32
    rng = np.random.default_rng(1)
    dev = torch.device("cuda", 0)
    from fmidx.sharding import payload_header_words

    H = payload_header_words(B)
    dense_rows = np.zeros((P, B, W), dtype=np.uint32)
    pays = []
    wide = rng.random(B) < args.wide
    for p in range(P):
        desc = np.zeros(B, dtype=np.uint32)
        off = np.zeros(B, dtype=np.uint32)
        data = []
        at = H
        for b in range(B):
            if wide[b] or rng.random() < args.dense:
                bits = (rng.random(W * 32) < 0.1).astype(np.uint8)
                bits[V:] = 0
                row = np.packbits(bits, bitorder="little").view(np.uint32)
                dense_rows[p, b] = row
                desc[b] = W | 0x80000000
            else:
                k = int(rng.geometric(1.0 / args.mean)) - 1
                toks = rng.integers(0, V, size=k)
                row = (toks + SH).astype(np.uint32)
                np.bitwise_or.at(dense_rows[p, b], toks // 32, (1 << (toks % 32)).astype(np.uint32))
                desc[b] = k
            pad = (-row.size) % 4
            off[b] = at
            data.append(np.concatenate([row, np.zeros(pad, dtype=np.uint32)]))
            at += row.size + pad
        head = np.zeros(H, dtype=np.uint32)
        head[:4] = [at, B, W, 0x58534D46]
        head[4:4 + B] = desc
        head[4 + B:4 + 2 * B] = off
        pays.append(np.concatenate([head] + data))
    m = max(x.size for x in pays)
    sp = np.zeros((P, m), dtype=np.uint32)
    for p, x in enumerate(pays):
        sp[p, :x.size] = x
    sp_t = torch.from_numpy(sp.view(np.int32)).to(dev)
    dn_t = torch.from_numpy(dense_rows.view(np.int32)).to(dev)
    out_s = torch.empty((B, V), dtype=torch.uint8, device=dev)
    out_d = torch.empty((B, V), dtype=torch.uint8, device=dev)
    or_payloads(sp_t, B, V, SH, out=out_s)
    or_bits(dn_t, V, out=out_d)
    torch.cuda.synchronize()
    exact = bool(torch.equal(out_s, out_d))
    K = args.K
    flush = torch.zeros(1 << 28, dtype=torch.int32, device=dev)

    def timed(fn, src):
        cp = src.unsqueeze(0).expand(K, *src.shape).contiguous()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for i in range(K):
                fn(cp[i])
        res = {}
        for mode in ("warm", "cold"):
            ts = []
            for _ in range(3):
                if mode == "cold":
                    flush.add_(1)
                torch.cuda.synchronize()
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                g.replay()
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) / K * 1e3)
            res[mode] = float(np.median(ts))
        return res

    r_s = timed(lambda x: or_payloads(x, B, V, SH, out=out_s), sp_t)
    r_d = timed(lambda x: or_bits(x, V, out=out_d), dn_t)
    print(json.dumps({"exact": exact,
                      "payload_bytes": int(sum(x.size for x in pays) * 4), "dense_bytes": int(dense_rows.nbytes),
                      "or_rows_us": r_s, "or_bits_us": r_d}), flush=True)


if __name__ == "__main__":
    main()
