"""Device known answers: the trace kernel's own primitive code (rfx.h rfx_kat_*) against the outputs the
unmodified reference computed for the same inputs (tests/golden/kat_*.npz, tools/gen_golden.py):

* Sphere::trace / Triangle::trace (untextured, bilinear-textured, checker-textured) / Plane::trace with and
  without out-parameters (Sphere.cpp:44-85, Triangle.cpp:53-108, Plane.cpp:36-73) on seeded rays built to hit
  the edge cases -- inside-sphere origins, surface +- DELTA, tangents, rays pointing away, zero rays, the radius
  clamp, barycentric edges, near-degenerate and parallel triangles, origins on a vertex, parallel planes;
* Skybox::getTexelColor (checker and atlas) on the 6 faces, edges, corners, the zero ray;
* Texture::getTexelColor(u, v) on the [0, 1] boundaries and 1 - FLT_EPSILON (32- and 24-bpp TGA texels);
* powf at both Scene.cpp call sites' domains (glibc 2.35, kat_pow.npz) and Color::argb.

Bar: bit-exact (0 ULP on every output float).
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN
from reflaxman_amd.render import DIELECTRIC, METAL, Color, Material, Renderer, Scene, Vector3

pytestmark = pytest.mark.gpu

KAT_MAT = Material(METAL, Color(0.25, 0.5, 0.75), 0.5, 0.0)  # oracle/ref_harness.cpp kat_material


def load(key):
    return np.load(os.path.join(GOLDEN, key + ".npz"))


def run_objects(scene, rays, n):
    r = Renderer()
    r.set_scene(scene)
    out = r.kat_objects(rays, np.arange(n, dtype=np.int32))
    r.close()
    return out


def assert_same(out, ref, key):
    bad = np.argwhere(out.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, f"{key}: {len(bad)} values differ, first {bad[:5].tolist()}"


def test_kat_sphere():
    g = load("kat_sphere")
    rec = g["inp"]
    s = Scene()
    for q in rec:
        s.addSphere(Vector3(*q[6:9]), float(q[9]), KAT_MAT)
    out = run_objects(s, rec[:, :6], rec.shape[0])
    assert g["out"][:, 0].sum() > 100 and g["out"][:, 14].sum() > 100
    assert_same(out, g["out"], "kat_sphere")


@pytest.mark.parametrize("key,texture", [("kat_triangle", "none"), ("kat_triangle_tex", "tex"),
                                         ("kat_triangle_checker", "empty")])
def test_kat_triangle(key, texture):
    g = load(key)
    rec = g["inp"]
    s = Scene()
    tex = None
    if texture != "none":
        tex = s.addTextureArgb(g["tex"] if texture == "tex" else None)
    for q in rec:
        t = s.addTriangle(Vector3(*q[6:9]), Vector3(*q[9:12]), Vector3(*q[12:15]), KAT_MAT)
        if tex is not None:
            t.setTexture(tex, *[float(v) for v in q[15:21]])
    out = run_objects(s, rec[:, :6], rec.shape[0])
    assert g["out"][:, 0].sum() > 100
    assert_same(out, g["out"], key)


def test_kat_plane():
    g = load("kat_plane")
    rec = g["inp"]
    s = Scene()
    for q in rec:
        s.addPlane(Vector3(*q[6:9]), Vector3(*q[9:12]), KAT_MAT)
    out = run_objects(s, rec[:, :6], rec.shape[0])
    assert g["out"][:, 0].sum() > 100
    assert_same(out, g["out"], "kat_plane")


def test_kat_mixed_objects_one_scene():
    """Spheres, triangles and planes in ONE scene (the object map through the Morton sphere order)."""
    gs, gt, gp = load("kat_sphere"), load("kat_triangle"), load("kat_plane")
    s = Scene()
    rays, objs, ref = [], [], []
    n = 300
    for i in range(n):
        a, b, c = gs["inp"][i], gt["inp"][i], gp["inp"][i]
        objs.append(s.addSphere(Vector3(*a[6:9]), float(a[9]), KAT_MAT).obj); rays.append(a[:6]); ref.append(gs["out"][i])
        objs.append(s.addTriangle(Vector3(*b[6:9]), Vector3(*b[9:12]), Vector3(*b[12:15]), KAT_MAT).obj)
        rays.append(b[:6]); ref.append(gt["out"][i])
        objs.append(s.addPlane(Vector3(*c[6:9]), Vector3(*c[9:12]), KAT_MAT).obj); rays.append(c[:6]); ref.append(gp["out"][i])
    r = Renderer()
    r.set_scene(s)
    perm = np.random.default_rng(5).permutation(len(objs))
    out = r.kat_objects(np.array(rays)[perm], np.array(objs, np.int32)[perm])
    r.close()
    assert_same(out, np.array(ref)[perm], "mixed")


@pytest.mark.parametrize("key,skybox", [("kat_skybox_checker", False), ("kat_skybox_tex", True)])
def test_kat_skybox(key, skybox):
    g = load(key)
    s = Scene()
    if skybox:
        s.setSkyboxTextureArgb(g["tex"])
    r = Renderer()
    r.set_scene(s)
    out = r.kat_texels(-1, g["inp"])
    r.close()
    assert_same(out, g["out"], key)


@pytest.mark.parametrize("key,textured", [("kat_texture_checker", False), ("kat_texture_tex", True),
                                          ("kat_texture_tex24", True)])
def test_kat_texture(key, textured):
    g = load(key)
    s = Scene()
    s.addTextureArgb(g["tex"] if textured else None)
    r = Renderer()
    r.set_scene(s)
    out = r.kat_texels(0, g["inp"])
    r.close()
    assert_same(out, g["out"], key)


def test_kat_powf():
    g = load("kat_pow")
    r = Renderer()
    out = r.kat_powf(g["inp"])
    r.close()
    assert_same(out, g["out"], "kat_pow")


def test_kat_powf_cube_every_float():
    """The Fresnel site's powf(x, 3) (Scene.cpp:196) takes the double cube where it provably rounds like glibc: on
    the device it equals glibc's algorithm for every float in [0, 1] (tests/test_powf.py checks the host copy against
    the live libm on the same floats)."""
    r = Renderer()
    bad, slow = r.kat_powf_cube()
    r.close()
    assert bad == 0
    assert 0 < slow < 0x3f800001


def test_kat_division_fast_path():
    """The trace loop's division fast path (rfx_math.h: eight of the IEEE lowering's eleven instructions, for divisors
    in [2^-40, 2^100] and quotients in [2^-60, 2^60]; the shared-reciprocal form of Vector3 / float) equals IEEE '/'
    bit for bit on 2^27 + 2^20 operand pairs (5 quotients each: div_rn, normalize's three, the skybox's): raw bit patterns of every class, both edges of both
    bounds, zero and denormal numerators (tests/test_div_guard.py replays the range argument on the CPU)."""
    import ctypes as C
    from reflaxman_amd import _lib
    r = Renderer()
    counts = (C.c_uint64 * 3)()
    _lib.check(_lib.load().rfx_kat_div(r._h, 0, (1 << 27) + (1 << 20), counts), "kat_div")
    r.close()
    bad, fast, seen = counts
    assert seen == 5 * ((1 << 27) + (1 << 20))
    assert bad == 0
    # the fast path is taken on most of the in-range classes and refused on the rest (NaN, zero, out-of-range pairs)
    assert 0.2 * (seen // 5) < fast < 0.99 * (seen // 5), fast


def test_kat_argb():
    g = load("kat_argb")
    r = Renderer()
    out = r.kat_argb(g["inp"])
    r.close()
    assert np.array_equal(out, g["out"])


def test_triangle_reject_before_divide_decides_like_the_divide():
    """Large-scene shadow rays reject plane crossings outside a triangle before the correctly rounded divide
    (rfx_trace.h tri_hit PRE); the KAT kernel evaluates both forms and writes NaN where they disagree.  2^20 rays
    aimed within a few ulp of the edges u = 0, v = 0, u + v = 1 (and at random points), from random origins and
    ray lengths: no disagreement."""
    rng = np.random.default_rng(7)
    n = 1 << 20
    s = Scene()
    quads = [((-5.0, 0.0, -5.0), (5.0, 0.0, -5.0), (5.0, 0.0, 5.0)), ((-5.0, 0.0, -5.0), (5.0, 0.0, 5.0), (-5.0, 0.0, 5.0)),
             ((-3.0, -2.0, 7.0), (4.0, 1.5, 7.5), (0.5, 6.0, 8.0))]
    for a, b, c in quads:
        s.addTriangle(Vector3(*a), Vector3(*b), Vector3(*c), KAT_MAT)
    obj = rng.integers(0, len(quads), n).astype(np.int32)
    v0 = np.array([q[0] for q in quads], np.float64)[obj]
    e1 = (np.array([q[1] for q in quads], np.float64) - np.array([q[0] for q in quads]))[obj]
    e2 = (np.array([q[2] for q in quads], np.float64) - np.array([q[0] for q in quads]))[obj]
    u = rng.random(n)
    v = rng.random(n) * (1 - u)
    eps = rng.normal(0, 1e-6, n)
    edge = rng.integers(0, 4, n)
    u = np.where(edge == 0, eps, u)
    v = np.where(edge == 1, eps, v)
    v = np.where(edge == 2, 1 - u + eps, v)
    p = v0 + u[:, None] * e1 + v[:, None] * e2
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    o = p + d * rng.uniform(0.01, 50.0, n)[:, None]
    ray = (p - o) * rng.uniform(0.05, 20.0, n)[:, None]
    rays = np.concatenate([o, ray], axis=1).astype(np.float32)
    r = Renderer()
    r.set_scene(s)
    out = r.kat_objects(rays, obj)
    r.close()
    assert not np.isnan(out[:, 14]).any(), int(np.isnan(out[:, 14]).sum())
    assert 0.2 * n < out[:, 14].sum() < 0.9 * n  # both outcomes well represented


@pytest.mark.parametrize("scene_name", ["default", "stress4096"])
def test_kernarg_layout(scene_name):
    """The bounce loops read the scene record and the frame parameters through the kernarg segment pointer
    (rfx_trace.h launder_scene / kernarg_params), assuming DevScene at offset 0 and FrameParams after it.  A kernel of
    the trace kernels' signature finds every word of both equal to its by-value arguments; one declared with the two
    arguments swapped finds differences, so the check would catch a kernel whose signature moved them."""
    import ctypes as C
    from reflaxman_amd import _lib, scenes
    from reflaxman_amd.render import build_scene
    scene, _ = build_scene(scenes.get_scene(scene_name))
    r = Renderer()
    r.set_scene(scene)
    L = _lib.load()
    good, swapped = (C.c_uint32 * 3)(), (C.c_uint32 * 3)()
    _lib.check(L.rfx_kat_kernarg(r._h, 0, good), "kat_kernarg")
    _lib.check(L.rfx_kat_kernarg(r._h, 1, swapped), "kat_kernarg")
    assert list(good) == [0, 0, 1], list(good)  # (1: this build reads the record laundered)
    assert swapped[0] > 0 and swapped[1] > 0, list(swapped)
    r.close()
