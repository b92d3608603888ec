"""Exactness of the RNG pre-pass's divide-free component (rfx_math.h rand_component_dev).

Vector3::randomInsideSphere computes ``float(k) / (float(FAST_RAND_MAX) / 2) - 1.f``
(reference src/common/Vector3.cpp:182-184) with k = fastrand() in [0, 0x7FFF].
The host replaces the f32 divide by ``(float)((double)k * (1.0 / 16383.5))`` and the device
pre-pass by an f32 product with one fma fix-up; this checks, for all 32768 possible k, that
each rounds to the reference's float.
"""
from fractions import Fraction

import numpy as np


def test_rand_component_divide_free_is_exact_for_every_k():
    k = np.arange(0x8000, dtype=np.uint32)
    ref = k.astype(np.float32) / np.float32(np.float32(0x7FFF) / np.float32(2.0)) - np.float32(1.0)
    dev = (k.astype(np.float64) * (1.0 / 16383.5)).astype(np.float32) - np.float32(1.0)
    assert ref.dtype == dev.dtype == np.float32
    assert np.array_equal(ref.view(np.uint32), dev.view(np.uint32))


def test_rand_component_fma_fixup_is_exact_for_every_k():
    """Device form: q = k*r, e = fma(-q, d, k), fma(e, r, q), r = f32(1/d), d = 16383.5 -- each fma
    emulated exactly (the products fit a double; the final sum is rounded once, via Fraction)."""
    k = np.arange(0x8000, dtype=np.uint32).astype(np.float32)
    d = np.float32(16383.5)
    r = np.float32(1.0) / d
    ref = k / d
    q = k * r
    e = (k.astype(np.float64) - q.astype(np.float64) * np.float64(d)).astype(np.float32)  # exact, then one rounding
    fr = Fraction(float(r))
    for i in range(0x8000):
        exact = Fraction(float(e[i])) * fr + Fraction(float(q[i]))
        got = np.float32(float(exact))  # Fraction -> double is exact-to-nearest; check it lands on ref's float
        lo = np.nextafter(ref[i], np.float32(-np.inf))
        hi = np.nextafter(ref[i], np.float32(np.inf))
        dist = abs(exact - Fraction(float(ref[i])))
        assert dist <= abs(exact - Fraction(float(lo))) and dist <= abs(exact - Fraction(float(hi))), i
        assert got == ref[i] or dist == abs(exact - Fraction(float(got))), i
