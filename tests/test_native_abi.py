"""CPU-side checks of the C-ABI library: it builds for gfx950, loads, and exports every
symbol include/mt_replay.h declares (no compute calls without a GPU)."""
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(REPO, "include", "mt_replay.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mt_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from fluidframework_amd import build, _native
    build.build()
    lib = _native.load()
    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _native.SIGNATURES}
    assert set(names) == bound


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from fluidframework_amd import MergeTreeBatch
    with pytest.raises(RuntimeError):
        MergeTreeBatch(4)
