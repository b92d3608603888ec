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


K_TAKE_BELOW = F32(float.fromhex("0x1.ffffep-1"))  # rfx_trace.h kTakeBelow = 1 - 2^-20
K_TAKE_ABOVE = F32(float.fromhex("0x1.00001p+0"))  # rfx_trace.h kTakeAbove = 1 + 2^-20


def test_take_band_orders_rounded_distances():
    """rfx_trace.h sph_takes / tri_takes decide outside a 2^-20 band around best_sq without square roots:
    sq < RN(best_sq (1 - 2^-20)) must give sqrt_rn(sq) < sqrt_rn(best_sq), sq > RN(best_sq (1 + 2^-20)) must give
    sqrt_rn(sq) > sqrt_rn(best_sq).  Checked at the band's edges (the floats just outside it) for best_sq over the
    normal range of squared distances, every significand pattern near binade edges included."""
    rng = np.random.default_rng(7)
    best = np.concatenate([
        (rng.uniform(-27.0, 40.0, 400000)).astype(np.float64),
    ])
    best = np.exp2(best).astype(F32)
    # binade edges: 1, succ(1), pred(2) ... scaled over the range
    edge = np.array([1.0, 1.0000001, 1.9999999, 1.5, 1.4142135], np.float64)
    best = np.concatenate([best, (edge[None, :] * np.exp2(np.arange(-27, 40))[:, None]).astype(F32).ravel()])
    best = best[np.isfinite(best) & (best > 0)]
    lo = (best * K_TAKE_BELOW).astype(F32)
    hi = (best * K_TAKE_ABOVE).astype(F32)
    below = np.nextafter(lo, F32(0), dtype=F32)           # largest sq with sq < lo
    above = np.nextafter(hi, F32(np.inf), dtype=F32)      # smallest sq with sq > hi
    rb = np.sqrt(best)
    assert np.all(np.sqrt(below) < rb)
    assert np.all(np.sqrt(above) > rb)
    # also a spread of candidates inside the fast regions
    for f in (0.5, 0.9, 0.99999, 0.999999):
        sq = (best * F32(f)).astype(F32)
        m = sq < lo
        assert np.all(np.sqrt(sq[m]) < rb[m])
    for f in (1.000002, 1.00001, 1.5):
        sq = (best * F32(f)).astype(F32)
        m = np.isfinite(sq) & (sq > hi)
        assert np.all(np.sqrt(sq[m]) > rb[m])
