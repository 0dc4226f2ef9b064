"""Summarise tools/pmc_traffic.sh output into profiles/pmc_traffic.json form:
per-launch HBM bytes of the fused decode kernel (the last K eager
k_decode<false, true> dispatches = the timed steps replayed eagerly)."""
import csv
import hashlib
import json
import os
import sys

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fm-index-constrained-decoding_amd", "fmidx",
                   "libfmidx.so")


def lib_sha16(path=LIB):
    """The first 16 hex digits of the SHA-256 of the library the counters were
    collected with: bench.py uses the committed figure only for the same build."""
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def per_dispatch(path, counter, kernel="k_decode<false, true,"):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if kernel not in name or r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    steps = int(args[args.index("--steps") + 1]) if "--steps" in args else 20
    bench = json.load(open(os.path.join(out, "bench_FETCH_SIZE.json")))
    fetch = per_dispatch(os.path.join(out, "counters_FETCH_SIZE.csv"), "FETCH_SIZE")[-steps:]
    write = per_dispatch(os.path.join(out, "counters_WRITE_SIZE.csv"), "WRITE_SIZE")[-steps:]
    fb = 2 * 1024 * sum(fetch) / len(fetch)
    wb = 1024 * sum(write) / len(write)
    # the standalone LF kernel: the last K k_lf dispatches (eager replay)
    lf_fetch = per_dispatch(os.path.join(out, "counters_FETCH_SIZE.csv"), "FETCH_SIZE", "k_lf")[-steps:]
    lf_write = per_dispatch(os.path.join(out, "counters_WRITE_SIZE.csv"), "WRITE_SIZE", "k_lf")[-steps:]
    lfb = (2 * 1024 * sum(lf_fetch) / len(lf_fetch) + 1024 * sum(lf_write) / len(lf_write)) if lf_fetch else None
    res = {
        "kernel": "k_decode<false, true> (fused LF step + uint8 mask)",
        "lib_sha16": lib_sha16(),
        "corpus_tokens": bench["config"]["corpus_tokens"],
        "batch": bench["config"]["batch_per_gpu"],
        "dispatches": [len(fetch), len(write)],
        "fetch_bytes_per_launch": fb,
        "write_bytes_per_launch": wb,
        "k_decode_bytes_per_launch": fb + wb,
        "alg_bytes_per_launch": bench["roofline"]["alg_bytes_per_launch"],
        "k_lf_bytes_per_launch": lfb,
        "k_lf_alg_bytes_per_launch": bench["standalone_kernels"]["k_lf"]["alg_bytes_per_launch"],
        "correction": "bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE "
                      "counts half of wide coalesced reads; counters in KB)",
    }
    print(json.dumps(res, indent=1))
    with open(os.path.join(out, "pmc_traffic.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
