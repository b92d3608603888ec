"""The division fast path's range argument (rfx_math.h div_prep / div_fast), replayed in float32 on the CPU.

gfx950 lowers a correctly rounded f32 a / b as v_div_scale (b), v_div_scale (a), v_rcp, six fma/mul steps, v_div_fmas
and v_div_fixup.  The device fast path runs only the eight middle instructions, which is the same computation whenever
both v_div_scale are identities (no rescale, VCC clear) and v_div_fixup only re-applies the quotient's own sign.  The
guard admits a quotient when the divisor b lies in [2^-40, 2^100] and the fast quotient q' in [2^-60, 2^60].  This
test restates the ISA's conditions for a rescale or a special fixup (the CDNA ISA's V_DIV_SCALE_F32 / V_DIV_FIXUP_F32
pseudo-code) and checks that no (a, b) the guard admits meets any of them -- at the corners of the guarded region, with
q' anywhere within 8 ulps of the true quotient (the fast sequence is within a few ulps), and on random pairs.  The
device side (the eight instructions against '/') is checked by tests/test_gpu_kat.py::test_kat_division_fast_path."""
import numpy as np

B_LO, B_HI, Q_LO, Q_HI = 2.0 ** -40, 2.0 ** 100, 2.0 ** -60, 2.0 ** 60
F32_MIN = 2.0 ** -126


def f32(x):
    return np.float32(x)


def biased_exp(x) -> int:
    return int((np.float32(x).view(np.uint32) >> 23) & 0xFF)


def rescale_or_special(a, b) -> list:
    """The conditions under which v_div_scale does not return its operand unchanged with VCC clear, or v_div_fixup
    does more than apply sign(a) ^ sign(b) to |q2| (operands as float32)."""
    a, b = f32(a), f32(b)
    why = []
    if not (np.isfinite(a) and np.isfinite(b)):
        why.append("nan/inf operand")
        return why
    if a == 0 or b == 0:
        why.append("zero operand")
        return why
    ea, eb = biased_exp(a), biased_exp(b)
    if ea - eb >= 96:
        why.append("exponent(a) - exponent(b) >= 96")
    if eb == 0:
        why.append("b denormal")
    inv = 1.0 / float(b)
    if abs(inv) < F32_MIN:
        why.append("1/b denormal")
    qa = float(a) / float(b)
    if abs(qa) < F32_MIN:
        why.append("a/b denormal")
    if ea <= 23:
        why.append("exponent(a) <= 23")
    if ea - eb < -150:
        why.append("fixup underflow")
    if eb == 255 or ea == 255:
        why.append("fixup overflow")
    return why


def admitted(b, qfast) -> bool:
    return B_LO <= abs(float(b)) <= B_HI and Q_LO <= abs(float(qfast)) <= Q_HI


def ulps(x, k):
    """x moved by k ulps (float32)."""
    u = np.float32(x).view(np.int32)
    return np.int32(u + k).view(np.float32)


def test_corners_of_the_guarded_region():
    """Divisors and fast quotients at and just inside both bounds; numerators a = q b with q up to 8 ulps away from
    the fast quotient in either direction (and their float32 neighbours)."""
    checked = 0
    for b0 in (B_LO, B_HI):
        for db in (-2, -1, 0, 1, 2):
            b = ulps(f32(b0), db)
            for q0 in (Q_LO, Q_HI, 1.0):
                for dq in (-3, 0, 3):
                    qf = ulps(f32(q0), dq)
                    if not admitted(b, qf):
                        continue
                    for err in range(-8, 9):  # the true quotient within 8 ulps of the fast one
                        q = ulps(qf, err)
                        for sb in (1.0, -1.0):
                            for sq in (1.0, -1.0):
                                a = f32(float(q) * sq * float(b) * sb)
                                if not np.isfinite(a):  # no finite numerator has this quotient (q b > 2^128)
                                    continue
                                for da in (-1, 0, 1):
                                    aa = ulps(a, da)
                                    assert rescale_or_special(aa, f32(float(b) * sb)) == [], (aa, b, qf)
                                    checked += 1
    assert checked > 1000


def test_random_admitted_pairs():
    """1e6 random pairs over the whole float32 range: every pair the guard admits (with the exact quotient standing in
    for the fast one, and its 4-ulp neighbours) meets none of the conditions."""
    rng = np.random.default_rng(1234)
    n = 1_000_000
    bits_a = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    # divisors mostly in and around the guarded range, numerators anywhere
    eb = rng.integers(127 - 50, 127 + 110, n).astype(np.uint32)
    bits_b = (rng.integers(0, 2, n).astype(np.uint32) << 31) | (eb << 23) | rng.integers(0, 1 << 23, n).astype(np.uint32)
    a = bits_a.view(np.float32)
    b = bits_b.view(np.float32)
    with np.errstate(all="ignore"):
        q = (a.astype(np.float64) / b.astype(np.float64)).astype(np.float32)
    seen = 0
    for k in (-4, 0, 4):
        qf = (q.view(np.int32) + np.int32(k)).view(np.float32)
        with np.errstate(invalid="ignore"):
            ok = (np.abs(b) >= B_LO) & (np.abs(b) <= B_HI) & (np.abs(qf) >= Q_LO) & (np.abs(qf) <= Q_HI)
        idx = np.flatnonzero(ok)
        seen += idx.size
        # vectorised restatement of rescale_or_special on the admitted pairs
        aa, bb = a[idx], b[idx]
        ea = (aa.view(np.uint32) >> 23) & 0xFF
        ebb = (bb.view(np.uint32) >> 23) & 0xFF
        qa = aa.astype(np.float64) / bb.astype(np.float64)
        bad = (~np.isfinite(aa)) | (aa == 0) | (ea.astype(np.int64) - ebb >= 96) | (ebb == 0) | \
              (np.abs(1.0 / bb.astype(np.float64)) < F32_MIN) | (np.abs(qa) < F32_MIN) | (ea <= 23) | \
              (ea.astype(np.int64) - ebb < -150) | (ea == 255) | (ebb == 255)
        assert not bad.any(), (aa[bad][:4], bb[bad][:4])
        # and the scalar restatement agrees on a sample
        for i in idx[:200]:
            assert rescale_or_special(a[i], b[i]) == []
    assert seen > 100_000


def test_the_conditions_do_fire_outside_the_region():
    """The restated conditions are live: pairs just outside the guard meet them where the ISA rescales."""
    assert "exponent(a) <= 23" in rescale_or_special(f32(2.0 ** -110), f32(1.0))
    assert "a/b denormal" in rescale_or_special(f32(2.0 ** -100), f32(2.0 ** 40))
    assert "1/b denormal" in rescale_or_special(f32(1.0), f32(2.0 ** 127))
    assert "exponent(a) - exponent(b) >= 96" in rescale_or_special(f32(2.0 ** 60), f32(2.0 ** -40))
    assert "zero operand" in rescale_or_special(f32(0.0), f32(3.0))
    assert "b denormal" in rescale_or_special(f32(1e-30), f32(1e-40))
