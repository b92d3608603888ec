"""Exactness of the RNG pre-pass's divide-free component (rfx_math.h rand_component_dev).

Vector3::randomInsideSphere computes ``float(k) / (float(FAST_RAND_MAX) / 2) - 1.f``
(reference src/common/Vector3.cpp:182-184) with k = fastrand() in [0, 0x7FFF].
The device pre-pass replaces the f32 divide by ``(float)((double)k * (1.0 / 16383.5))``;
this checks, for all 32768 possible k, that the two round to the same float.
"""
import numpy as np


def test_rand_component_divide_free_is_exact_for_every_k():
    k = np.arange(0x8000, dtype=np.uint32)
    ref = k.astype(np.float32) / np.float32(np.float32(0x7FFF) / np.float32(2.0)) - np.float32(1.0)
    dev = (k.astype(np.float64) * (1.0 / 16383.5)).astype(np.float32) - np.float32(1.0)
    assert ref.dtype == dev.dtype == np.float32
    assert np.array_equal(ref.view(np.uint32), dev.view(np.uint32))
