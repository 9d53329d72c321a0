"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/svo_gpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import numpy as np

import svo_amd as S
import svo_amd.scene as SC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="svo_gpu.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
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


def test_synth_library_is_separate_from_the_product():
    """The synthetic workload generator (include/svo_synth.h) lives in its own
    test/bench library; the product library exports none of it."""
    assert set(declared_symbols("svo_synth.h")) == set(SC.SYNTH_SYMBOLS)
    syn = ctypes.CDLL(SC.synth_lib_path())
    gpu = ctypes.CDLL(S.lib_path())
    for name in SC.SYNTH_SYMBOLS:
        assert hasattr(syn, name) and not hasattr(gpu, name), name


def test_synth_is_deterministic_host_code():
    a = SC.synth_canvas(3, 200, 100, 50)
    b = SC.synth_canvas(3, 200, 100, 50)
    assert np.array_equal(a, b) and a.std() > 10
    K = np.array([[100, 0, 100], [0, 100, 50], [0, 0, 1]], np.float64)
    f = SC.synth_frame(a, (20, 20), np.eye(3), K, 1, 3, 160, 60)
    assert f.shape == (60, 160)


def test_tracking_library_exports_every_declared_symbol():
    from svo_amd import tracking as T
    assert set(declared_symbols("svo_tracking.h")) == set(T.SYMBOLS)
    lib = ctypes.CDLL(T.lib_path())
    for name in declared_symbols("svo_tracking.h"):
        assert hasattr(lib, name), name


def test_tracking_create_fails_loudly_without_device():
    """No HIP device here: the host mirror refuses to run instead of falling back."""
    import pytest
    from svo_amd import tracking as T
    if S.lib().svo_ctx_create(0, ctypes.byref(ctypes.c_void_p())) == 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(S.SvoError):
        T.Tracking(np.zeros(24, np.float32))


def test_stereo_synth_is_consistent_with_depth_field():
    """Right view of the synthetic rig: a left pixel's disparity is bf / z of its surface point."""
    from svo_amd.scene import Scene, STEREO_BF
    sc = Scene(320, 240, seed=5)
    L, R = sc.frame(0), sc.right(0)
    assert L.shape == R.shape and abs(int(L.mean()) - int(R.mean())) < 3
    X = sc.map_points(np.array([[160.0, 120.0]]), 0)
    d = STEREO_BF / X[0, 2]
    # SAD over a patch is minimal at the predicted disparity (integer search)
    y, x = 120, 160
    patch = L[y - 6:y + 7, x - 6:x + 7].astype(int)
    sad = [np.abs(R[y - 6:y + 7, x - k - 6:x - k + 7].astype(int) - patch).sum() for k in range(0, 40)]
    assert abs(int(np.argmin(sad)) - d) <= 1.0


def test_host_pool_runs_every_task_exactly_once():
    """The front end's host pool (frontend.cpp Pool) under its real pattern: jobs of
    sizes that change every round (one RANSAC hypothesis per task) with primes
    between them. A worker left over from an older job must never claim a task
    of a newer one (the claim word carries generation and count together)."""
    for threads in (2, 5, 16):
        assert S.pool_selftest(threads, 4000) == 0, threads
