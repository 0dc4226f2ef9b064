"""Index-structure options and launch tuning (include/fmidx.h: fm_build_options,
fm_tuning) -- the engine's construction surface beside the reference's
(cpp_modules_linux/fm_index.hpp:20-45 has one layout: sdsl's csa_wt_int<>).

    from fmidx import options
    ix = FMIndex(options=options.build_options("compact"))          # 54 GiB at C3
    ix = FMIndex(options=options.build_options(cache_min=8, bm_log2=6))
    with options.tuning(lf_group=4, lf_work=0):                     # process-wide, restored on exit
        ...

The environment carries at most two override strings for measurement runs,
FMIDX_BUILD_OPTIONS and FMIDX_TUNING ("key=value,...", keys = field names).
"""
from __future__ import annotations

import contextlib
import ctypes
from ctypes import c_int32, c_uint32, c_uint64
from typing import Optional, Union

from ._lib import check, lib

PROFILES = {"default": 0, "compact": 1}


class BuildOptions(ctypes.Structure):
    """fm_build_options."""
    _fields_ = [("size", c_uint32), ("profile", c_int32), ("transitions", c_int32), ("lf_e", c_int32),
                ("lf_e2", c_int32), ("probe_first", c_int32), ("keep_bwt", c_int32), ("follow_bitmaps", c_int32),
                ("bm_log2", c_int32), ("trans_min", c_int32), ("cache_min", c_uint64), ("cache_mb", c_uint64),
                ("trans_mb", c_uint64), ("gpu_sort_min", c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k not in ("size", "reserved")}


class Tuning(ctypes.Structure):
    """fm_tuning."""
    _fields_ = [("size", c_uint32), ("lf_group", c_uint32), ("search_group", c_uint32), ("dec_threads", c_uint32),
                ("mask_slices", c_uint32), ("reserved", c_uint32), ("lf_group_min", c_uint64), ("lf_work", c_int32),
                ("lf_gprobe", c_int32), ("lf_quad", c_int32), ("lf_split", c_int32), ("search_p8", c_int32),
                ("reserved2", c_int32), ("lf_sweep_min", c_uint64), ("sa_chunk", c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("reserved") and k != "size"}


assert ctypes.sizeof(BuildOptions) == 72 and ctypes.sizeof(Tuning) == 72


def build_options(profile: Union[str, int] = "default", **fields) -> BuildOptions:
    """A profile's options (fm_build_options_init) with ``fields`` changed."""
    p = PROFILES[profile] if isinstance(profile, str) else int(profile)
    o = BuildOptions()
    check(lib().fm_build_options_init(ctypes.byref(o), p), "build_options_init")
    for k, v in fields.items():
        if k in ("size", "reserved", "profile") or not hasattr(o, k):
            raise TypeError(f"build_options: unknown field {k!r}")
        setattr(o, k, int(v))
    return o


def as_build_options(options) -> Optional[BuildOptions]:
    """None, a BuildOptions, a profile name or a dict (with an optional "profile")."""
    if options is None or isinstance(options, BuildOptions):
        return options
    if isinstance(options, (str, int)):
        return build_options(options)
    if isinstance(options, dict):
        d = dict(options)
        return build_options(d.pop("profile", "default"), **d)
    raise TypeError(f"options: a BuildOptions, profile name or dict, not {type(options).__name__}")


def get_tuning() -> Tuning:
    t = Tuning()
    check(lib().fm_get_tuning(ctypes.byref(t)), "get_tuning")
    return t


def set_tuning(t: Optional[Tuning] = None, **fields) -> Tuning:
    """Process-wide launch tuning: ``t`` (default: the current one) with
    ``fields`` changed.  Returns the tuning in force before."""
    old = get_tuning()
    new = Tuning()
    ctypes.memmove(ctypes.byref(new), ctypes.byref(t if t is not None else old), ctypes.sizeof(Tuning))
    for k, v in fields.items():
        if k.startswith("reserved") or k == "size" or not hasattr(new, k):
            raise TypeError(f"tuning: unknown field {k!r}")
        setattr(new, k, int(v))
    check(lib().fm_set_tuning(ctypes.byref(new)), "set_tuning")
    return old


def default_tuning() -> Tuning:
    t = Tuning()
    check(lib().fm_tuning_init(ctypes.byref(t)), "tuning_init")
    return t


@contextlib.contextmanager
def tuning(**fields):
    """with tuning(lf_group=4): ... -- the launch tuning changed for the block."""
    old = set_tuning(**fields)
    try:
        yield
    finally:
        check(lib().fm_set_tuning(ctypes.byref(old)), "set_tuning")


__all__ = ["BuildOptions", "Tuning", "build_options", "as_build_options", "get_tuning", "set_tuning",
           "default_tuning", "tuning", "PROFILES"]
