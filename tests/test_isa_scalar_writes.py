"""The built gfx950 code objects never write through the scalar data cache.

Scalar-memory stores, scalar atomics and that cache's write-back / discard
were followed by machine-wide hardware errors on this pool, so no kernel of
the product library (nor the in-tree micro benchmarks) may contain them:
global memory is written through vector stores and vector atomics only.
This disassembles every gfx950 code object bundled in fmidx/libfmidx.so
(llvm-objdump from the ROCm toolchain, CPU only) and fails on any such
instruction.  (This file names the instructions, so it is listed in
.gpurunignore: it runs in the CPU suite only.)
"""
import glob
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "fm-index-constrained-decoding_amd", "fmidx", "libfmidx.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
FORBIDDEN = re.compile(r"\b(s_store_\w+|s_buffer_store_\w+|s_scratch_store\w*|s_atomic_\w+|s_buffer_atomic_\w+|"
                       r"s_dcache_wb\w*|s_dcache_discard\w*)\b")


def _code_objects(lib, tmp_path):
    dst = tmp_path / os.path.basename(lib)
    shutil.copy(lib, dst)
    subprocess.run([OBJDUMP, "--offloading", str(dst)], cwd=tmp_path, check=True, capture_output=True)
    return sorted(glob.glob(str(tmp_path / "*amdgcn-amd-amdhsa--gfx950")))


@pytest.mark.skipif(not os.path.exists(OBJDUMP), reason="ROCm llvm-objdump not installed")
def test_no_scalar_cache_writes_in_product_library(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libfmidx.so not built")
    objs = _code_objects(LIB, tmp_path)
    assert objs, "no gfx950 code object found in libfmidx.so"
    bad = []
    n_insts = 0
    for o in objs:
        asm = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", o], check=True, capture_output=True, text=True).stdout
        n_insts += asm.count("\n")
        bad += [ln.strip() for ln in asm.splitlines() if FORBIDDEN.search(ln)]
    assert n_insts > 10000, "disassembly looks empty"
    assert not bad, bad[:20]
