"""Drop-in replacement for the reference's SWIG package ``cpp_modules``.

Putting ``fm-index-constrained-decoding_amd/`` on ``sys.path`` makes the
reference's own ``index.py`` (``from cpp_modules.fm_index import FMIndex as
_FMIndex, load_FMIndex``) run unchanged on the MI355X engine.
"""
