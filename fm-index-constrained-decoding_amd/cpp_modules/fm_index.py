"""``cpp_modules.fm_index`` (reference: SWIG module ``fm_index``, fm_index.i:7)
backed by libfmidx.so.  Exposes exactly the SWIG names: ``FMIndex`` and
``load_FMIndex`` (fm_index.hpp:20-45)."""
from fmidx.fm_index import FMIndex, load_FMIndex  # noqa: F401

__all__ = ["FMIndex", "load_FMIndex"]
