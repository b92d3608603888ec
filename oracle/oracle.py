"""ORACLE TEST INFRASTRUCTURE -- ctypes binding of oracle/_ref/liboracle.so.

The CPU restatement of ReflaxMan's trace loop (rfx_oracle.c), used only as
the checker by tests/, ``__graft_entry__.smoke()`` and the ``cpu_baseline``
leg of bench.py.  Never imported by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_ref", "liboracle.so")
REFHARNESS = os.path.join(HERE, "_ref", "refharness")

COUNTER_NAMES = [
    "rays", "segments",
    "sph_tests", "sph_b", "sph_d", "sph_t",
    "tri_tests", "tri_z", "tri_s", "tri_t", "tri_in", "tri_d",
    "hit_sph", "hit_tri",
    "sh_sph_tests", "sh_sph_b", "sh_sph_d", "sh_sph_t",
    "sh_tri_tests", "sh_tri_z", "sh_tri_s", "sh_tri_t", "sh_tri_in",
    "l_eval", "l_facing", "l_lit", "l_spec", "l_pow",
    "dielectric", "metal", "continue", "sky",
    "tex_bilinear", "tex_checker", "tex_other",
    "pln_tests", "pln_t", "hit_pln", "sh_pln_tests", "sh_pln_t",
]

_fp = C.POINTER(C.c_float)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB):
        subprocess.run(["make", "-C", HERE, "port"], check=True, capture_output=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        L.orc_scene_new.restype = C.c_void_p
        L.orc_scene_new.argtypes = [C.c_float] * 4
        L.orc_scene_free.argtypes = [C.c_void_p]
        L.orc_add_texture.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, _u32p]
        L.orc_set_skybox.argtypes = [C.c_void_p, C.c_int]
        L.orc_add_light.argtypes = [C.c_void_p, _fp, C.c_float, _fp, C.c_float]
        L.orc_add_sphere.argtypes = [C.c_void_p, _fp, C.c_float, C.c_int, _fp, C.c_float, C.c_float]
        L.orc_add_triangle.argtypes = [C.c_void_p, _fp, _fp, _fp, C.c_int, _fp, C.c_float, C.c_float]
        L.orc_add_plane.argtypes = [C.c_void_p, _fp, _fp, C.c_int, _fp, C.c_float, C.c_float]
        L.orc_triangle_set_texture.argtypes = [C.c_void_p, C.c_int, C.c_int, _fp]
        L.orc_camera_view.argtypes = [_fp, _fp, _fp]
        L.orc_render.argtypes = [C.c_void_p, _fp, _fp, C.c_float, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                 C.c_int, C.c_int, _u32p, _u32p, _fp, C.c_int, _u64p]
        L.orc_render_band.argtypes = [C.c_void_p, _fp, _fp, C.c_float, C.c_uint32, C.c_uint32, C.c_int,
                                      C.c_uint32, C.c_uint32, C.c_uint32, _fp, _u32p, C.c_int, _u64p]
        L.orc_rand_dirs.argtypes = [_u32p, C.c_uint64, _fp]
        L.orc_kat_sphere.argtypes = [_fp, C.c_uint64, _fp]
        L.orc_kat_triangle.argtypes = [_fp, C.c_uint64, C.c_uint32, C.c_uint32, _u32p, C.c_int, _fp]
        L.orc_kat_plane.argtypes = [_fp, C.c_uint64, _fp]
        L.orc_kat_skybox.argtypes = [C.c_uint32, C.c_uint32, _u32p, _fp, C.c_uint64, _fp]
        L.orc_kat_texture.argtypes = [C.c_uint32, C.c_uint32, _u32p, _fp, C.c_uint64, _fp]
        L.orc_argb.restype = C.c_uint32
        L.orc_argb.argtypes = [C.c_float] * 3
        _lib = L
    return _lib


def _f(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a, a.ctypes.data_as(_fp)


def _u(a):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    return a, a.ctypes.data_as(_u32p)


class OracleScene:
    """Scene built through the restatement's builder calls, in SceneDesc order."""

    def __init__(self, desc):
        L = lib()
        self.desc = desc
        self.h = C.c_void_p(L.orc_scene_new(*desc.diffuse))
        self._keep = []
        if desc.skybox is not None and desc.skybox.argb is not None:
            t, p = _u(desc.skybox.argb)
            self._keep.append(t)
            L.orc_set_skybox(self.h, L.orc_add_texture(self.h, desc.skybox.width, desc.skybox.height, p))
        for (o, r, c, pw) in desc.lights:
            L.orc_add_light(self.h, _f(o)[1], r, _f(c)[1], pw)
        tex_ids = []
        for t in desc.textures:
            if t.argb is None:
                tex_ids.append(L.orc_add_texture(self.h, 0, 0, None))
            else:
                a, p = _u(t.argb)
                tex_ids.append(L.orc_add_texture(self.h, t.width, t.height, p))
        for ob in desc.objects:
            mt, rgb, refl, tr = ob[-1]
            if ob[0] == "sphere":
                L.orc_add_sphere(self.h, _f(ob[1])[1], ob[2], mt, _f(rgb)[1], refl, tr)
            elif ob[0] == "plane":
                L.orc_add_plane(self.h, _f(ob[1])[1], _f(ob[2])[1], mt, _f(rgb)[1], refl, tr)
            else:
                L.orc_add_triangle(self.h, _f(ob[1])[1], _f(ob[2])[1], _f(ob[3])[1], mt, _f(rgb)[1], refl, tr)
        for (oi, ti, uv) in desc.settex:
            L.orc_triangle_set_texture(self.h, oi, tex_ids[ti], _f(uv)[1])
        eye, at, fov = desc.camera
        self.eye = np.array(eye, np.float32)
        self.view = camera_view(eye, at)
        self.fov = fov

    def __del__(self):
        try:
            lib().orc_scene_free(self.h)
        except Exception:
            pass


def camera_view(eye, at) -> np.ndarray:
    v = np.zeros(9, np.float32)
    lib().orc_camera_view(_f(eye)[1], _f(at)[1], v.ctypes.data_as(_fp))
    return v


class OracleRender:
    """Render-shaped driver over the restatement (Render.cpp:57-226 semantics)."""

    def __init__(self, desc, sphere_seed=1350490027, jitter_seed=0):
        self.scene = OracleScene(desc)
        self.sphere_seed = C.c_uint32(sphere_seed)
        self.jitter_seed = C.c_uint32(jitter_seed)
        self.additive_counter = 0
        self.image = None
        self.W = self.H = 0

    def set_image_size(self, W, H):
        self.W, self.H = W, H
        self.image = np.zeros((H, W, 3), np.float32)
        self.additive_counter = 0

    def render(self, depth, ss, additive=False, nthreads=1, counters=None):
        self.additive_counter = self.additive_counter + 1 if additive else 0
        cnt = None if counters is None else counters.ctypes.data_as(_u64p)
        rc = lib().orc_render(self.scene.h, self.scene.eye.ctypes.data_as(_fp), self.scene.view.ctypes.data_as(_fp),
                              self.scene.fov, self.W, self.H, depth, ss, int(bool(additive)), self.additive_counter,
                              C.byref(self.sphere_seed), C.byref(self.jitter_seed),
                              self.image.ctypes.data_as(_fp), nthreads, cnt)
        if rc != 0:
            raise ValueError("orc_render rejected its arguments")

    def image_pixels(self) -> np.ndarray:
        """Render::imagePixel for every pixel (divides by additiveCounter when > 1)."""
        if self.additive_counter > 1:
            return (self.image / np.float32(self.additive_counter)).astype(np.float32)
        return self.image.copy()

    def argb(self) -> np.ndarray:
        """Render::copyImage (no division, Render.cpp:82-101)."""
        return argb_of(self.image)


def argb_of(img: np.ndarray) -> np.ndarray:
    """Color::argb over an (..., 3) float32 array: trunc(c * 255.999f) low byte per channel."""
    q = img.astype(np.float32) * np.float32(255.999)
    b = np.where(q < 2.0 ** 31, q, 0).astype(np.int64) & 0xFF  # cvttss2si + low byte
    return ((b[..., 0] << 16) | (b[..., 1] << 8) | b[..., 2]).astype(np.uint32)


def render_band(desc, W, H, depth, y0, rows, sphere_seed=1350490027, nthreads=1, counters=None):
    sc = OracleScene(desc)
    rgb = np.zeros((rows, W, 3), np.float32)
    argb = np.zeros((rows, W), np.uint32)
    cnt = None if counters is None else counters.ctypes.data_as(_u64p)
    rc = lib().orc_render_band(sc.h, sc.eye.ctypes.data_as(_fp), sc.view.ctypes.data_as(_fp), sc.fov, W, H, depth,
                               y0, rows, sphere_seed, rgb.ctypes.data_as(_fp), argb.ctypes.data_as(_u32p), nthreads, cnt)
    if rc != 0:
        raise ValueError("orc_render_band rejected its arguments")
    return rgb, argb


def rand_dirs(seed, n):
    s = C.c_uint32(seed)
    out = np.zeros((n, 3), np.float32)
    lib().orc_rand_dirs(C.byref(s), n, out.ctypes.data_as(_fp))
    return out, s.value


def kat(kind, rec, tex=None, textured=False):
    L = lib()
    rec, p = _f(rec)
    n = rec.shape[0]
    if kind == "sphere":
        out = np.zeros((n, 15), np.float32); L.orc_kat_sphere(p, n, out.ctypes.data_as(_fp))
    elif kind == "plane":
        out = np.zeros((n, 15), np.float32); L.orc_kat_plane(p, n, out.ctypes.data_as(_fp))
    elif kind == "triangle":
        out = np.zeros((n, 15), np.float32)
        if tex is None:
            L.orc_kat_triangle(p, n, 0, 0, None, int(textured), out.ctypes.data_as(_fp))
        else:
            t, tp = _u(tex)
            L.orc_kat_triangle(p, n, t.shape[1], t.shape[0], tp, int(textured), out.ctypes.data_as(_fp))
    elif kind == "skybox":
        out = np.zeros((n, 3), np.float32)
        if tex is None:
            L.orc_kat_skybox(0, 0, None, p, n, out.ctypes.data_as(_fp))
        else:
            t, tp = _u(tex)
            L.orc_kat_skybox(t.shape[1], t.shape[0], tp, p, n, out.ctypes.data_as(_fp))
    elif kind == "texture":
        out = np.zeros((n, 3), np.float32)
        if tex is None:
            L.orc_kat_texture(0, 0, None, p, n, out.ctypes.data_as(_fp))
        else:
            t, tp = _u(tex)
            L.orc_kat_texture(t.shape[1], t.shape[0], tp, p, n, out.ctypes.data_as(_fp))
    else:
        raise ValueError(kind)
    return out
