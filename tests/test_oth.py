"""``.oth`` metadata (index.py:189-207): the reference pickles the tuple
(beginnings, occurring, labels); fmidx reads such files with an unpickler
that resolves no globals, and still reads its own earlier JSON files."""
import json
import os
import pickle

import pytest

from fmidx.index import read_oth


def test_reads_reference_pickle(tmp_path):
    p = str(tmp_path / "x.oth")
    meta = ([0, 3, 7], [5, 1, 9], ["a", "b"])
    with open(p, "wb") as f:
        pickle.dump(meta, f)                 # exactly index.py:194
    assert read_oth(p) == ([0, 3, 7], [5, 1, 9], ["a", "b"])
    for proto in range(0, pickle.HIGHEST_PROTOCOL + 1):
        with open(p, "wb") as f:
            pickle.dump(([0, 2], {4, 6}, None), f, protocol=proto)   # a set (as before index.py:54) / no labels
        b, o, lab = read_oth(p)
        assert b == [0, 2] and set(o) == {4, 6} and lab is None


def test_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    p = str(tmp_path / "evil.oth")
    with open(p, "wb") as f:
        pickle.dump(([0, 1], [Evil()], None), f)
    with pytest.raises(pickle.UnpicklingError):
        read_oth(p)


def test_reads_legacy_json(tmp_path):
    p = str(tmp_path / "j.oth")
    with open(p, "w") as f:
        json.dump({"beginnings": [0, 4], "occurring": [3, 2], "labels": None}, f)
    assert read_oth(p) == ([0, 4], [3, 2], None)
