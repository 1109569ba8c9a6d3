"""The counter RNG: committed golden vectors, the oracle and the device
library's host implementation (rt_rng_u32) agree; basic uniformity."""
import json
import os

import numpy as np

import oracle
from rt_amd import abi

CASES = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "rng_vectors.json")))["cases"]


def test_golden_vectors_oracle_and_library_agree():
    lib = abi.load()
    for seed, pixel, sample, dim, want in CASES:
        assert oracle.rng_u32(seed, pixel, sample, dim) == want
        assert lib.rt_rng_u32(seed, pixel, sample, dim) == want


def test_draws_are_distinct_across_samples_of_a_pixel():
    lib = abi.load()
    for dim in (0, 3, 15):
        v = {lib.rt_rng_u32(1, 1234, s, dim) for s in range(4096)}
        assert len(v) == 4096  # a bijection in the sample index for a fixed (pixel, dim)


def test_uniformity():
    lib = abi.load()
    u = np.array([lib.rt_rng_u32(5, p, s, d) >> 8 for p in range(16) for s in range(64) for d in range(20)],
                 dtype=np.float64) / 2 ** 24
    assert abs(u.mean() - 0.5) < 0.01
    hist, _ = np.histogram(u, bins=16, range=(0, 1))
    chi2 = ((hist - len(u) / 16) ** 2 / (len(u) / 16)).sum()
    assert chi2 < 45  # 15 degrees of freedom, p ~ 1e-4
