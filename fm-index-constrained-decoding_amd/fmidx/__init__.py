"""MI355X-native FM-index engine for document-constrained decoding.

``fmidx.fm_index.FMIndex``  -- SWIG surface (cpp_modules_linux/fm_index.hpp)
``fmidx.index.FMIndex``     -- index.py surface (index.py:20-207)
``fmidx.processors``        -- batched logits processors (document_constrained_generation_*)
"""
from ._lib import FMIndexError, LIB_PATH  # noqa: F401

__all__ = ["FMIndexError", "LIB_PATH"]
