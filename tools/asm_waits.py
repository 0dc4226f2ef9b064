"""Find loads that go out one round trip at a time in the device assembly.

Compiles a .hip file to gfx950 assembly and, per kernel, lists every place
where a vector-memory load is followed by a full wait (s_waitcnt vmcnt(0) or
lgkmcnt(0) after a FLAT load) before the next load is issued.  A dependent
chain (a rank block, then the BWT word it points to) looks the same and is
expected; a run of such waits over independent loads (an unrolled batch whose
loads sit under branches, FLAT loads through a pointer handed over in LDS) is
a serialised batch and costs a round trip per load.

Usage: python tools/asm_waits.py csrc/decode.hip [kernel-substring] [-v]
"""
import os
import re
import subprocess
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fm-index-constrained-decoding_amd")
# .loc file numbers: see the .file directives of the listing
LOAD = re.compile(r"\t(global_load|buffer_load|flat_load|scratch_load)\w*")


def kernels(asm):
    lines = asm.split("\n")
    starts = [(i, l[:-1].split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    for i, name in starts:
        end = next(j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end"))
        yield name, lines[i:end]


def serialised(body):
    """(line, load, wait, next load) for load -> full wait -> load."""
    out = []
    last_load = None
    waited = None
    loc = "?"
    for i, l in enumerate(body):
        if l.strip().startswith(";"):
            continue
        if l.strip().startswith(".loc\t"):
            f = l.split()
            loc = f"{f[1]}:{f[2]}"
            continue
        m = LOAD.match(l)
        if m:
            if last_load is not None and waited is not None:
                out.append((last_load[2], last_load[1].strip(), waited.strip(), l.strip() + "  @" + loc))
            last_load = (i, l, loc)
            waited = None
        elif last_load is not None and ("s_waitcnt vmcnt(0)" in l or
                                        ("flat_load" in last_load[1] and "lgkmcnt(0)" in l)):
            waited = l
        elif l.startswith(".LBB") or "s_cbranch" in l or "s_branch" in l:
            pass
    return out


def main():
    src = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else ""
    verbose = "-v" in sys.argv
    out = "/tmp/asm_waits.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                    "-mllvm", "-amdgpu-kernarg-preload-count=7", "-gline-tables-only", "-x", "hip", "--offload-device-only", "-S",
                    os.path.join(PKG, src) if not os.path.isabs(src) else src, "-o", out], check=True)
    asm = open(out).read()
    for name, body in kernels(asm):
        if pat not in name:
            continue
        s = serialised(body)
        nl = sum(1 for l in body if LOAD.match(l))
        nf = sum(1 for l in body if "\tflat_load" in l)
        print(f"{name[:90]}: {nl} loads, {nf} flat, {len(s)} load->wait->load")
        if verbose:
            for ln, a, w, b in s:
                print(f"    @{ln:8s} {a[:40]:40s} | {w[:20]:20s} | {b[:40]} {b[b.rfind('@'):]}")


if __name__ == "__main__":
    main()
