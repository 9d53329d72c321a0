"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/svo_gpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import numpy as np

import svo_amd as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "svo_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(svo_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_what_python_binds():
    assert set(declared_symbols()) == set(S.SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(S.lib_path())
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_version_string():
    assert S.lib().svo_version().decode().startswith("svo_gpu gfx950")


def test_synth_is_deterministic_host_code():
    a = S.synth_canvas(3, 200, 100, 50)
    b = S.synth_canvas(3, 200, 100, 50)
    assert np.array_equal(a, b) and a.std() > 10
    K = np.array([[100, 0, 100], [0, 100, 50], [0, 0, 1]], np.float64)
    f = S.synth_frame(a, (20, 20), np.eye(3), K, 1, 3, 160, 60)
    assert f.shape == (60, 160)
