"""ctypes binding of ``libfmidx.so`` (C-ABI declared in ``include/fmidx.h``).

The library is built in-tree (``make -C fm-index-constrained-decoding_amd``)
and loaded from this directory.  There is no fallback: if the library is
missing, or no HIP device is present when an index is created, the error is
raised to the caller.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int64, c_size_t, c_uint8, c_uint32, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMIDX_LIB", os.path.join(HERE, "libfmidx.so"))

u64p = POINTER(c_uint64)
i64p = POINTER(c_int64)

# name -> (restype, argtypes); mirrors include/fmidx.h one to one
SIGNATURES = {
    "fm_last_error": (c_char_p, []),
    "fm_device_info": (c_int, [c_int, c_char_p, c_size_t]),
    "fm_create": (c_int, [POINTER(c_void_p), c_int]),
    "fm_destroy": (None, [c_void_p]),
    "fm_initialize": (c_int, [c_void_p, u64p, c_uint64]),
    "fm_initialize_from_file": (c_int, [c_void_p, c_char_p, c_int]),
    "fm_initialize_from_bwt_device": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "fm_initialize_from_text_device": (c_int, [c_void_p, c_void_p, c_uint64, c_int, c_void_p]),
    "fm_suffix_sort_device": (c_int, [c_void_p, c_uint64, c_void_p, c_void_p, c_void_p]),
    "fm_wt_int_levels_device": (c_int, [c_void_p, c_uint64, c_uint32, c_void_p, c_void_p]),
    "fm_size": (c_int, [c_void_p, u64p]),
    "fm_sigma": (c_int, [c_void_p, u64p]),
    "fm_backward_search_step": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, u64p]),
    "fm_backward_search_multi": (c_int, [c_void_p, u64p, c_uint64, u64p]),
    "fm_distinct": (c_int, [c_void_p, c_uint64, c_uint64, u64p, c_uint64, u64p]),
    "fm_distinct_count": (c_int, [c_void_p, c_uint64, c_uint64, u64p, c_uint64, u64p]),
    "fm_distinct_count_multi": (c_int, [c_void_p, u64p, u64p, c_uint64, u64p, c_uint64, u64p]),
    "fm_get_range_batch": (c_int, [c_void_p, i64p, i64p, c_uint64, c_int64, u64p, u64p, u64p, u64p]),
    "fm_locate": (c_int, [c_void_p, c_uint64, u64p]),
    "fm_extract_text": (c_int, [c_void_p, c_uint64, c_uint64, u64p, c_uint64, u64p]),
    "fm_save": (c_int, [c_void_p, c_char_p]),
    "fm_load": (c_int, [POINTER(c_void_p), c_char_p, c_int]),
    "fm_load_ex": (c_int, [POINTER(c_void_p), c_char_p, c_int, c_void_p]),
    "fm_build_options_init": (c_int, [c_void_p, c_int]),
    "fm_set_build_options": (c_int, [c_void_p, c_void_p]),
    "fm_get_build_options": (c_int, [c_void_p, c_void_p]),
    "fm_tuning_init": (c_int, [c_void_p]),
    "fm_set_tuning": (c_int, [c_void_p]),
    "fm_get_tuning": (c_int, [c_void_p]),
    "fm_lf_step_batch": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                 c_void_p, c_uint64, c_void_p]),
    "fm_backward_search_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_int64, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p]),
    "fm_allowed_mask_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_uint64,
                                      c_uint64, c_int64, c_int, c_void_p]),
    "fm_decode_step_batch": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_int, c_void_p]),
    "fm_distinct_count_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_uint64,
                                        c_void_p, c_void_p, c_void_p, c_void_p]),
    "fm_apply_boosts": (c_int, [c_int, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_void_p,
                                c_uint64, c_void_p, c_void_p, c_int64, c_void_p]),
    "fm_stats": (c_int, [c_void_p, u64p, u64p, u64p, u64p, u64p]),
    "fm_stats_ex": (c_int, [c_void_p, u64p, u64p, u64p, u64p, u64p]),
    "fm_stats_trans": (c_int, [c_void_p, u64p, u64p, u64p]),
    "fm_stats_trans_complete": (c_int, [c_void_p, POINTER(c_uint32)]),
    "fm_stats_mem": (c_int, [c_void_p, u64p, u64p, u64p]),
    "fm_locate_batch": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "fm_extract_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "fm_cache_lookup_batch": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]),
    "fm_processor_step": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_uint64, c_uint64, c_void_p, c_uint64,
                                  c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p]),
    "fm_processor_call": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "fm_shard_payload_capacity": (c_int, [c_uint64, c_uint64, u64p]),
    "fm_decode_step_payload": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p,
                                       c_void_p]),
    "fm_decode_step_payload_signal": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_void_p, c_void_p,
                                              c_void_p, c_uint64, c_void_p, c_void_p]),
    "fm_shard_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_void_p,
                              c_uint64, c_void_p]),
    "fm_shard_or_rows": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_int64, c_void_p, c_uint64,
                                 c_int, c_void_p]),
    "fm_shard_or_rows_peers": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_int64, c_void_p,
                                       c_uint64, c_int, c_void_p]),
    "fm_peer_signal": (c_int, [c_void_p, c_uint64, c_void_p, c_void_p]),
    "fm_lf_persist_status": (c_int, [c_void_p, POINTER(c_uint32)]),
    "fm_shard_or_rows_peers_wait": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_int64, c_void_p,
                                            c_uint64, c_int, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p]),
    "fm_shard_pack_facts": (c_int, [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p, c_uint64, c_uint64, c_void_p,
                                    c_void_p, c_uint64, c_void_p]),
    "fm_shard_or_rows_facts": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_int64, c_void_p, c_uint64,
                                       c_int, c_void_p, c_void_p]),
    "fm_shard_or_rows_peers_facts": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_int64, c_void_p,
                                             c_uint64, c_int, c_void_p, c_void_p, c_uint32, c_void_p, c_void_p,
                                             c_void_p]),
    "fm_peer_flags_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p]),
    "fm_host_mapped_alloc": (c_int, [c_uint64, POINTER(c_void_p)]),
    "fm_host_mapped_free": (c_int, [c_void_p]),
    "fm_ipc_handle": (c_int, [c_void_p, c_void_p, u64p]),
    "fm_ipc_open": (c_int, [c_void_p, POINTER(c_void_p)]),
    "fm_ipc_close": (c_int, [c_void_p]),
    "fm_processor_shard_prep": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "fm_processor_shard_finish": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]),
    "fm_or_bits": (c_int, [c_void_p, c_uint64, c_uint64, c_uint64, c_uint64, c_uint64, c_void_p, c_uint64, c_int,
                            c_void_p]),
    "fm_probe_gather": (c_int, [c_void_p, c_uint64, c_int, c_uint64, c_uint32, c_void_p, c_void_p]),
    "fm_device_bwt": (c_int, [c_void_p, POINTER(c_void_p)]),
    "fm_release_bwt_view": (c_int, [c_void_p]),
    "fm_stats_views": (c_int, [c_void_p, POINTER(c_uint64)]),
    "fm_device_struct": (c_int, [c_void_p, c_int, POINTER(c_void_p), POINTER(c_uint64)]),
    "fm_synchronize": (c_int, [c_void_p]),
    "fm_reload_tuning": (c_int, []),
    "fm_attach_isa_samples_device": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
}

_lib = None


class FMIndexError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load libfmidx.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FMIndexError(
                f"{LIB_PATH} not found: build it with `make -C fm-index-constrained-decoding_amd` "
                "(there is no CPU fallback)")
        dll = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                fn = getattr(dll, name)
            except AttributeError:
                # a measurement variant of another build (FMIDX_LIB, tools/ab_decode.py) may lack
                # newer entry points; the product library exports every one (tests/test_abi.py)
                if "FMIDX_LIB" not in os.environ:
                    raise
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = dll
    return _lib


def last_error() -> str:
    msg = lib().fm_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, what: str = "") -> int:
    if rc != 0:
        raise FMIndexError(f"{what or 'fmidx'} failed ({rc}): {last_error()}")
    return rc


def u64_array(values):
    arr = (c_uint64 * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr


def i64_array(values):
    arr = (c_int64 * max(1, len(values)))()
    for i, v in enumerate(values):
        arr[i] = v
    return arr


__all__ = ["lib", "check", "last_error", "FMIndexError", "u64_array", "i64_array", "SIGNATURES",
           "LIB_PATH", "c_uint8"]
