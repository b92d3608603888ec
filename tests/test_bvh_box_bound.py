"""The BVH box test (rfx_trace.h bvh_box, ray_inv) keeps every box a reported sphere hit can lie in.

A sphere the reference reports as hit lies within r + 1.25e-3 |o - c| of the ray (tests/test_cull_bound.py), so a ray
that reports a hit on a sphere inside a BVH child box passes within delta = 1.25e-3 (|o - centre| + half-diagonal) of
that box at some t > 0.  The kernel widens the box by m = kCullRel (|o - ref| + mt) + 1e-6 >= kCullRel (|o - centre| +
half-diagonal) + 1e-6 and runs the slab test in float32 with approximate reciprocals.  This test aims rays at points
inside the box grown by 0.95 delta -- from origins 0.05 .. 200 box sizes away, with unnormalised directions, some
axis-parallel -- and checks that the kernel's float arithmetic keeps every such box, in both forms: the unfused slab
((bound - m) - o) * rcp(d) and the fused one fma(bound - m, rcp(d), -(o * rcp(d))) (RFX_BVH_FMA).  The fused form needs
finite reciprocals: with rcp(0) = inf, inf - inf leaves one slab end NaN and fminf / fmaxf take the other end for both,
which culls axis-parallel rays that pass through the box (476 of 2^19 here before ray_inv clamped them to +-1e30).
"""
import numpy as np
import pytest

F = np.float32
K_CULL_REL = F(2e-3)  # rfx_trace.h kCullRel


def approx(x, rng, ulps=1.0):
    """A hardware approximation (v_rcp_f32 / v_sqrt_f32) within `ulps` ulp of the rounded value."""
    x = x.astype(F)
    return (x.astype(np.float64) * (1.0 + rng.uniform(-ulps, ulps, x.shape) * 2.0 ** -23)).astype(F)


def fmaf(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F)


def kept(lo, hi, o, d, ref, mt, rng, fused):
    """rfx_trace.h ray_inv + bvh_box for one child, in float32 (fused: False, True or "prewide")."""
    e = o - ref
    dm = K_CULL_REL * (approx(np.sqrt((e * e).sum(1, dtype=F)), rng) * F(1.0001)) + F(1e-6)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        inv = approx(F(1) / d, rng)
        if fused:  # ray_inv clamps the reciprocals to +-1e30 for the fused forms
            inv = np.clip(inv, F(-1e30), F(1e30))
        if fused == "prewide":
            # rfx_host.cpp: the box grown by kCullRel mt (x (1 + 1e-6)) and rounded outward; the kernel's slab
            # constants (o + dm) rcp(d) and (o - dm) rcp(d)
            w = 2e-3 * mt.astype(np.float64) * (1.0 + 1e-6)
            lo = np.nextafter((lo.astype(np.float64) - w[:, None]).astype(F), F(-np.inf))
            hi = np.nextafter((hi.astype(np.float64) + w[:, None]).astype(F), F(np.inf))
            a = fmaf(lo, inv, -((o + dm[:, None]) * inv))
            b = fmaf(hi, inv, -((o - dm[:, None]) * inv))
            mn, mx = np.fmin(a, b), np.fmax(a, b)
            t0 = np.fmax(np.fmax(mn[:, 0], mn[:, 1]), np.fmax(mn[:, 2], F(0)))
            t1 = np.fmin(np.fmin(mx[:, 0], mx[:, 1]), mx[:, 2])
            return ~(t0 > t1 * F(1.00001) + F(1e-30))
        elif fused:  # RFX_BVH_FMA without pre-widening (RFX_BVH_PREWIDE=0)
            m = fmaf(np.full_like(mt, K_CULL_REL), mt, dm)
            oi = o * inv
            a = fmaf(lo - m[:, None], inv, -oi)
            b = fmaf(hi + m[:, None], inv, -oi)
        else:
            m = dm + K_CULL_REL * mt
            a = (lo - m[:, None] - o) * inv
            b = (hi + m[:, None] - o) * inv
        # fminf / fmaxf: a NaN operand yields the other one
        mn, mx = np.fmin(a, b), np.fmax(a, b)
        t0 = np.fmax(np.fmax(mn[:, 0], mn[:, 1]), np.fmax(mn[:, 2], F(0)))
        t1 = np.fmin(np.fmin(mx[:, 0], mx[:, 1]), mx[:, 2])
        return ~(t0 > t1 * F(1.00001) + F(1e-30))


@pytest.mark.parametrize("fused", [False, True, "prewide"])
def test_box_test_keeps_every_box_a_reported_hit_lies_in(fused):
    rng = np.random.default_rng(20261017 + [False, True, "prewide"].index(fused))
    n = 1 << 19
    size = np.exp(rng.uniform(np.log(0.02), np.log(5.0), (n, 3)))         # half extents
    centre = rng.uniform(-20.0, 20.0, (n, 3))
    ref = centre + rng.uniform(-15.0, 15.0, (n, 3))                       # the BVH's reference point
    half_diag = np.linalg.norm(size, axis=1)
    mt = (np.linalg.norm(ref - centre, axis=1) + half_diag) * 1.0001      # host: nextafter up of mt * 1.0001
    mt = np.nextafter(mt.astype(F), F(np.inf))
    # a target inside the box grown by 0.95 delta, an origin 0.05 .. 200 box sizes away
    dist = half_diag * np.exp(rng.uniform(np.log(0.05), np.log(200.0), n))
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    o = centre + u * (half_diag + dist)[:, None]
    delta = 1.25e-3 * (np.linalg.norm(o - centre, axis=1) + half_diag)
    side = rng.uniform(-1.0, 1.0, (n, 3))
    face = rng.integers(0, 3, n)
    side[np.arange(n), face] = np.sign(side[np.arange(n), face])           # on a face of the grown box
    q = centre + side * (size + 0.95 * delta[:, None])
    d = (q - o) * np.exp(rng.uniform(np.log(0.1), np.log(30.0), n))[:, None]
    # every 16th ray axis-parallel in one coordinate (its origin moved onto the target's coordinate)
    ax = rng.integers(0, 3, n)
    par = np.arange(n) % 16 == 0
    o[par, ax[par]] = q[par, ax[par]]
    d[par, ax[par]] = 0.0
    # the moved origins change delta: check the rays whose target is still inside the box grown by 0.96 delta
    delta = 1.25e-3 * (np.linalg.norm(o - centre, axis=1) + half_diag)
    inside = (np.abs(q - centre) <= size + 0.96 * delta[:, None]).all(1)
    assert inside.sum() > n - n // 8
    lo, hi = (centre - size).astype(F), (centre + size).astype(F)
    k = kept(lo, hi, o.astype(F), d.astype(F), ref.astype(F), mt, rng, fused)
    assert k[inside].all(), int((~k[inside]).sum())


def test_entry_limit_keeps_what_the_product_form_keeps():
    """RFX_BVH_TLIM: a child is skipped when its entry parameter t0 exceeds tlim = sqrt(1.001 best / a) 1.0001 (approximate
    rcp and sqrt); the product form skips it when t0^2 a > 1.001 best.  Every child the product form keeps, tlim keeps."""
    rng = np.random.default_rng(7)
    n = 1 << 20
    a = np.exp(rng.uniform(np.log(1e-4), np.log(1e6), n)).astype(F)            # |ray|^2
    best = np.exp(rng.uniform(np.log(1e-8), np.log(1e8), n)).astype(F)         # best |ray t|^2 so far
    t0 = (np.sqrt(best.astype(np.float64) * 1.001 / a) * np.exp(rng.normal(0.0, 1e-5, n))).astype(F)
    keep_product = ~(t0 * t0 * a > best * F(1.001))
    tlim = approx(np.sqrt(best * F(1.001) * approx(F(1) / a, rng)), rng) * F(1.0001)
    keep_tlim = ~(t0 > tlim)
    assert keep_product.sum() > n // 4
    assert not (keep_product & ~keep_tlim).any()
