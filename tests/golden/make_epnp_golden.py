"""Writes tests/golden/epnp_host_64.npz: 64 five-point subsets (4 noise levels)
and the product's host EPnP outputs for them (R | t as float64 bits, ok flags).
Run from the repo root after building: python tests/golden/make_epnp_golden.py"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from test_epnp_cpu import host_epnp, subsets  # noqa: E402

subs = np.concatenate([subsets(10 + i, 16, noise)[0] for i, noise in enumerate((0.0, 0.3, 1.0, 5.0))])
Rt, ok = host_epnp(subs)
np.savez(os.path.join(HERE, "epnp_host_64.npz"), subsets=subs, Rt=Rt, ok=ok)
print("wrote", len(subs), "subsets; ok", int(ok.sum()))
