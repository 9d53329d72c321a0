"""Host time per 5-point subset of the RANSAC minimal solver in each form
(svo_epnp_subsets device 3 scalar / 4 AVX2 lanes / 5 AVX-512 lanes / 0 as
dispatched), single thread: python tools/epnp_isa_bench.py [M]"""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "tests")]
import svo_amd as S  # noqa: E402
from test_epnp_cpu import K, subsets  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
subs, _, _ = subsets(5, m, 0.3)
f32p, f64p, i32p = C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_int)
Rt = np.zeros((m, 12))
ok = np.zeros(m, np.int32)
for dev, name in ((3, "scalar"), (4, "avx2"), (5, "avx512"), (0, "dispatched")):
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        rc = S.lib().svo_epnp_subsets(None, subs.ctypes.data_as(f32p), m, K.ctypes.data_as(f64p), dev,
                                      Rt.ctypes.data_as(f64p), ok.ctypes.data_as(i32p))
        best = min(best, time.perf_counter() - t0)
    print(f"{name:10s} rc {rc:3d}  {best / m * 1e6:.3f} us/subset")
