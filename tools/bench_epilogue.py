"""tools/bench_epilogue.py -- the fused logits epilogue (`fm_apply_boosts`,
SURVEY §8f row 1) timed against HBM and against torch's own `scores + mask`.

Workload: B x V scores (f32 / bf16 / f16), a bit-packed allowed set per row
at ~1 % density (what `fm_decode_step_batch(packed=1)` hands over), the
all_unigrams bit row, and per-row parameters with the allowed, unigram and
eos rules on.  Per launch the kernel reads the scores (V * sz per row) and
the row's allowed bits (V / 8), the shared unigram row once (V / 8, L2
resident afterwards), and writes V * sz:

    algorithmic bytes = B * (2 * V * sz + V / 8) + V / 8

The reference's last op is `scores + mask` over a dense mask of the scores
dtype (document_constrained_generation_causal_qwen.py:214) -- 3 * V * sz per
row even before the mask is assembled; it is timed beside for scale.  The
result is checked bit for bit against that torch expression.

    python tools/bench_epilogue.py [--batch 256] [--vocab 128256] [--iters 50]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "fm-index-constrained-decoding_amd"))

from fmidx._lib import check, lib  # noqa: E402
from fmidx.processors import ROW_DTYPE, _DTYPE_CODE, _round  # noqa: E402

HBM_PEAK_GBS = 8000.0


def run(dtype, B, V, iters, dev):
    g = torch.Generator(device="cpu").manual_seed(7)
    sz = torch.tensor([], dtype=dtype).element_size()
    scores = torch.randn((B, V), generator=g).to(dtype).to(dev)
    out = torch.empty_like(scores)
    allowed = torch.rand((B, V), generator=g) < 0.01
    uni = torch.rand(V, generator=g) < 0.5
    W = (V + 31) // 32

    def pack(b):      # bool [.., V] -> int32 [.., W], little-endian bit order
        a = np.pad(b.numpy().astype(np.uint8), [(0, 0)] * (b.dim() - 1) + [(0, W * 32 - V)])
        return torch.from_numpy(np.packbits(a, axis=-1, bitorder="little").view(np.int32).copy())

    bits = pack(allowed).to(dev)
    ubits = pack(uni[None])[0].to(dev)
    eos = 2
    rows = np.zeros(B, dtype=ROW_DTYPE)
    rows["base"] = 0.0
    rows["v_dist"] = _round(10.0, dtype)
    rows["v_uni"] = _round(5.0, dtype)
    rows["v_eos"] = _round(2.5, dtype)
    rows["flags"] = 1 | 2 | 4
    rp = torch.from_numpy(rows.view(np.uint8).copy()).to(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def launch():
        check(lib().fm_apply_boosts(_DTYPE_CODE[dtype], ctypes.c_void_p(scores.data_ptr()),
                                    ctypes.c_void_p(out.data_ptr()), B, V, V, V,
                                    ctypes.c_void_p(bits.data_ptr()), W, ctypes.c_void_p(ubits.data_ptr()),
                                    ctypes.c_void_p(rp.data_ptr()), eos, ctypes.c_void_p(stream)), "apply_boosts")

    # the reference's mask, assembled as it does (full, unigrams, distinct, eos)
    mask = torch.zeros((B, V), dtype=dtype, device=dev)
    mask[:, uni.to(dev)] = float(rows["v_uni"][0])
    mask[allowed.to(dev)] = float(rows["v_dist"][0])
    mask[:, eos] = float(rows["v_eos"][0])
    want = scores + mask
    launch()
    torch.cuda.synchronize()
    iv = torch.int32 if sz == 4 else torch.int16
    exact = bool(torch.equal(out.view(iv), want.view(iv)))

    def timed(fn):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / iters * 1e3   # us per launch

    us = timed(launch)
    tmp = torch.empty_like(scores)
    torch_us = timed(lambda: torch.add(scores, mask, out=tmp))
    alg = B * (2 * V * sz + V // 8) + V // 8
    gbs = alg / (us * 1e-6) / 1e9
    return {"dtype": str(dtype).replace("torch.", ""), "batch": B, "vocab": V, "us_per_launch": us,
            "alg_bytes_per_launch": alg, "GBps": gbs, "frac": gbs / HBM_PEAK_GBS,
            "torch_scores_plus_mask_us": torch_us, "bit_exact_vs_torch": exact}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        print(json.dumps(run(dt, args.batch, args.vocab, args.iters, dev)), flush=True)


if __name__ == "__main__":
    main()
