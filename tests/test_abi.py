"""C-ABI surface (CPU): the library loads, exports every symbol declared in
include/fmidx.h, the ctypes table matches the header, and -- with no GPU --
creating an index fails loudly instead of falling back to a CPU path."""
import os
import re

import pytest

from conftest import REPO, gpu_available

HEADER = os.path.join(REPO, "include", "fmidx.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for required in ["fm_create", "fm_destroy", "fm_initialize", "fm_initialize_from_file", "fm_size",
                     "fm_backward_search_step", "fm_backward_search_multi", "fm_distinct",
                     "fm_distinct_count", "fm_distinct_count_multi", "fm_locate", "fm_extract_text",
                     "fm_save", "fm_load", "fm_lf_step_batch", "fm_allowed_mask_batch",
                     "fm_distinct_count_batch", "fm_decode_step_batch"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    from fmidx._lib import SIGNATURES, lib

    dll = lib()
    names = declared_functions()
    for name in names:
        assert hasattr(dll, name), name
    assert sorted(SIGNATURES) == names


def test_nm_exports_match_header():
    import subprocess

    from fmidx._lib import LIB_PATH

    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (fm_[a-z0-9_]+)", out)))
    assert exported == declared_functions()


@pytest.mark.skipif(gpu_available(), reason="only meaningful without a GPU")
def test_no_cpu_fallback_without_gpu():
    from fmidx._lib import FMIndexError
    from fmidx.fm_index import FMIndex

    with pytest.raises(FMIndexError):
        FMIndex(device=0)


def test_swig_argument_errors_before_device():
    from fmidx.fm_index import _u64, _u64_vec

    with pytest.raises(OverflowError):
        _u64(-1, "backward_search_step", 2)
    with pytest.raises(TypeError):
        _u64(1.5, "backward_search_step", 2)
    with pytest.raises(OverflowError):
        _u64_vec([1, -2], "initialize", 2)
    assert _u64_vec([1, 2, 3], "initialize", 2).tolist() == [1, 2, 3]


def test_encode_corpus_matches_reference_encoding():
    from fmidx.index import encode_corpus
    from oracle.fm_oracle import encode_corpus as oracle_encode

    docs = [[1, 2, 3], [], [5], [0, 9, 9]]
    data, beg, occ = encode_corpus(docs)
    d2, b2, o2 = oracle_encode(docs)
    assert data.tolist() == d2 and beg == b2 and occ == o2


def _header_struct_fields(name):
    import re

    hdr = open(os.path.join(REPO, "include", "fmidx.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), hdr, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        names = decl.split(None, 1)[1] if not decl.startswith("const") else decl.split(None, 2)[2]
        for n in names.split(","):
            n = n.strip().lstrip("*").strip()
            fields.append(re.sub(r"\[.*\]", "", n))
    return fields


def test_ctypes_structs_match_header():
    """The ctypes mirrors of fm_prep_config / fm_processor_args / fm_peer_step list the
    header's fields in the header's order (their sizes are asserted at import
    and in api.cpp)."""
    import fmidx.processors as P

    assert [f[0] for f in P._PrepConfig._fields_] == _header_struct_fields("fm_prep_config")
    assert [f[0] for f in P._ProcessorArgs._fields_] == _header_struct_fields("fm_processor_args")
    from fmidx.sharding import FmPeerStep

    assert [f[0] for f in FmPeerStep._fields_] == _header_struct_fields("fm_peer_step")
