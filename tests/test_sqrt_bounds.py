"""Exactness of the squared-distance tests the trace kernel uses instead of square roots.

The reference compares rounded distances, dist = sqrtf(sq) with sq = |ray * t|^2
(Sphere.cpp:61-64, Triangle.cpp:70-85, closest hit Scene.cpp:92-105).  The kernel
compares squares instead (rfx_math.h):

* ``sqrt_rn(sq) > DELTA``  <=>  ``sq >= kSqDeltaSphere``;
* ``sqrt_rn(sq) >= y``      <=>  ``sq >= sq_lower_bound(y)``, so ``dist < best`` for
  sq < best_sq is ``sq < sq_lower_bound(best)``.

numpy's float32 sqrt is correctly rounded, as the reference's sqrtf and the device's
IEEE lowering are; these tests restate sq_lower_bound and check both facts.
"""
import numpy as np

F32 = np.float32


def succ(f):
    return np.nextafter(F32(f), F32(np.inf), dtype=F32)


def pred(f):
    return np.nextafter(F32(f), F32(0), dtype=F32)


def sq_lower_bound(y):
    """rfx_math.h sq_lower_bound: smallest float x with sqrt_rn(x) >= y (y > 0 finite)."""
    m = (float(pred(y)) + float(y)) * 0.5
    m2 = m * m
    f = F32(m2)
    if float(f) <= m2:
        f = succ(f)
    return f


K_SQ_DELTA_SPHERE = F32(float.fromhex("0x1.5798fp-27"))  # rfx_math.h kSqDeltaSphere


def test_k_sq_delta_sphere_matches_the_definition():
    assert sq_lower_bound(succ(F32(1e-4))) == K_SQ_DELTA_SPHERE


def test_k_sq_delta_sphere_is_the_exact_threshold():
    # every float within 2^20 ulps of the threshold classifies as the reference's sqrtf(sq) > DELTA
    k = int(K_SQ_DELTA_SPHERE.view(np.uint32))
    xs = (np.arange(-(1 << 20), 1 << 20, dtype=np.int64) + k).astype(np.uint32).view(F32)
    assert np.array_equal(np.sqrt(xs) > F32(1e-4), xs >= K_SQ_DELTA_SPHERE)


def test_sq_lower_bound_random_and_binade_edges():
    rng = np.random.default_rng(7)
    ys = list(rng.uniform(1e-4, 1e4, 20000).astype(F32))
    ys += [F32(2.0) ** e for e in range(-40, 40)]          # powers of two: predecessor in the lower binade
    ys += [succ(F32(2.0) ** e) for e in range(-40, 40)]
    ys += [F32(1e-4), succ(F32(1e-4)), F32(3.4e18)]
    for y in ys:
        lb = sq_lower_bound(y)
        assert np.sqrt(lb) >= y, y
        assert np.sqrt(pred(lb)) < y, y


def test_strictly_closer_equals_rounded_distance_compare():
    rng = np.random.default_rng(11)
    a = rng.uniform(1e-3, 50.0, 20000).astype(F32)
    # many near-ties: b within a few ulps of a
    b = (a.view(np.uint32).astype(np.int64) + rng.integers(-6, 7, a.size)).astype(np.uint32).view(F32)
    for sq, best_sq in zip(a, b):
        ref = bool(np.sqrt(sq) < np.sqrt(best_sq))
        mine = bool(sq < best_sq and sq < sq_lower_bound(np.sqrt(best_sq)))
        assert ref == mine, (sq, best_sq)
