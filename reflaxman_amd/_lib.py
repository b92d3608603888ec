"""ctypes binding of librfx.so (include/rfx.h).

This is the only way the package reaches the renderer: there is no CPU
fallback.  If the HIP library is missing or fails to load, every entry point
raises -- the product path never silently degrades to a CPU trace.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _build

RFX_OK = 0
RFX_NCOUNTERS = 40
RFX_ABI_VERSION = 3
METAL, DIELECTRIC = 0, 1

_fp = C.POINTER(C.c_float)
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)


class RfxError(RuntimeError):
    pass


class Frame(C.Structure):
    """rfx_frame (include/rfx.h)."""
    _fields_ = [
        ("eye", C.c_float * 3), ("view", C.c_float * 9), ("fov", C.c_float),
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("reflect_num", C.c_int32), ("sample_num", C.c_int32),
        ("additive", C.c_int32), ("additive_counter", C.c_int32),
        ("row_block", C.c_uint32), ("rank", C.c_uint32), ("nranks", C.c_uint32),
        ("pixel_begin", C.c_uint64), ("pixel_end", C.c_uint64),
        ("span_begin", C.c_uint64), ("span_end", C.c_uint64),
    ]


# (name, restype, argtypes) for every symbol of include/rfx.h
SIGNATURES = [
    ("rfx_abi_version", C.c_int, []),
    ("rfx_last_error", C.c_char_p, []),
    ("rfx_build_options", C.c_int, []),
    ("rfx_scene_create", C.c_void_p, [C.c_float] * 4),
    ("rfx_scene_destroy", None, [C.c_void_p]),
    ("rfx_scene_add_sphere", C.c_int, [C.c_void_p, _fp, C.c_float, C.c_int, _fp, C.c_float, C.c_float]),
    ("rfx_scene_add_triangle", C.c_int, [C.c_void_p, _fp, _fp, _fp, C.c_int, _fp, C.c_float, C.c_float]),
    ("rfx_scene_add_plane", C.c_int, [C.c_void_p, _fp, _fp, C.c_int, _fp, C.c_float, C.c_float]),
    ("rfx_scene_plane_count", C.c_int, [C.c_void_p]),
    ("rfx_triangle_set_texture", C.c_int, [C.c_void_p, C.c_int, C.c_int, _fp]),
    ("rfx_scene_add_light", C.c_int, [C.c_void_p, _fp, C.c_float, _fp, C.c_float]),
    ("rfx_scene_add_texture_argb", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, _u32p]),
    ("rfx_scene_add_texture_file", C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_int)]),
    ("rfx_scene_set_skybox_file", C.c_int, [C.c_void_p, C.c_char_p]),
    ("rfx_scene_set_skybox_argb", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32, _u32p]),
    ("rfx_scene_counts", C.c_int, [C.c_void_p] + [C.POINTER(C.c_int)] * 4),
    ("rfx_camera_view", None, [_fp, _fp, _fp]),
    ("rfx_camera_rz", C.c_float, [C.c_uint32, C.c_float]),
    ("rfx_tga_load", C.c_int, [C.c_char_p, _u32p, _u32p, _u32p, C.c_size_t]),
    ("rfx_tga_save", C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, _u32p]),
    ("rfx_bmp_save", C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, _u32p]),
    ("rfx_argb_from_rgb", None, [_fp, C.c_size_t, _u32p]),
    ("rfx_renderer_create", C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    ("rfx_renderer_destroy", None, [C.c_void_p]),
    ("rfx_renderer_device", C.c_int, [C.c_void_p]),
    ("rfx_renderer_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rfx_renderer_set_scene", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rfx_renderer_set_rng", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    ("rfx_renderer_get_rng", C.c_int, [C.c_void_p, _u32p, _u32p]),
    ("rfx_strip_rows", C.c_uint32, [C.c_uint32] * 4),
    ("rfx_strip_row_to_y", C.c_uint32, [C.c_uint32] * 4),
    ("rfx_render_frame", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rfx_render_frame_host", C.c_int, [C.c_void_p, C.POINTER(Frame), _fp, _u32p, _u64p]),
    ("rfx_frame_rng_blocks", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_uint32, _u64p]),
    ("rfx_frame_rng_count", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("rfx_render_frame_counted", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rfx_render_frame_counted_ev", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_uint32, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rfx_frame_rng_emit", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rfx_render_frame_emitted", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]),
    ("rfx_frame_rng_discard", C.c_int, [C.c_void_p]),
    ("rfx_frame_rng_pending", C.c_int, [C.c_void_p, _u32p]),
    ("rfx_frame_rng_rewind", C.c_int, [C.c_void_p]),
    ("rfx_group_create", C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_int), C.c_int]),
    ("rfx_group_destroy", None, [C.c_void_p]),
    ("rfx_group_size", C.c_int, [C.c_void_p]),
    ("rfx_group_renderer", C.c_void_p, [C.c_void_p, C.c_int]),
    ("rfx_group_set_scene", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rfx_group_set_bands", C.c_int, [C.c_void_p, C.c_uint32, _u32p]),
    ("rfx_group_get_bands", C.c_int, [C.c_void_p, _u32p]),
    ("rfx_group_render_frame", C.c_int, [C.c_void_p, C.POINTER(Frame), C.c_void_p, C.c_void_p, C.c_void_p]),
    ("rfx_renderer_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("rfx_renderer_set_tile_order", C.c_int, [C.c_void_p, C.c_int]),
    ("rfx_renderer_set_prim_masks", C.c_int, [C.c_void_p, C.c_int]),
    ("rfx_renderer_set_regroup", C.c_int, [C.c_void_p, C.c_int]),
    ("rfx_renderer_set_regroup_sort", C.c_int, [C.c_void_p, C.c_int]),
    ("rfx_renderer_set_launch_traces", C.c_int, [C.c_void_p, C.c_uint64]),
    ("rfx_renderer_bounce_form", C.c_int, [C.c_void_p]),
    ("rfx_renderer_get_timing", C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double), _u64p]),
    ("rfx_device_alloc", C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_void_p)]),
    ("rfx_device_free", C.c_int, [C.c_void_p, C.c_void_p]),
    ("rfx_memcpy_d2h", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rfx_memcpy_h2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rfx_memcpy_d2d", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    ("rfx_synchronize", C.c_int, [C.c_void_p]),
    ("rfx_rand_dirs", C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, _fp, _u32p]),
    ("rfx_kat_objects", C.c_int, [C.c_void_p, _fp, C.POINTER(C.c_int32), C.c_uint64, _fp]),
    ("rfx_kat_texels", C.c_int, [C.c_void_p, C.c_int, _fp, C.c_uint64, _fp]),
    ("rfx_kat_powf", C.c_int, [C.c_void_p, _fp, C.c_uint64, _fp]),
    ("rfx_kat_argb", C.c_int, [C.c_void_p, _fp, C.c_uint64, _u32p]),
    ("rfx_kat_powf_cube", C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    ("rfx_kat_div", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    ("rfx_kat_kernarg", C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_uint32)]),
]

_lib = None


def lib_path() -> str:
    return _build.LIB


def bind(path: str, partial: bool = False):
    """Load and bind any build of librfx.so (e.g. a variant build for A/B timing).  partial: an older build (tools/
    build_rev.py) may lack entry points added since; those are left unbound instead of failing."""
    L = C.CDLL(os.path.abspath(path))
    for name, res, args in SIGNATURES:
        if partial and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def load(build_if_missing: bool = True):
    """Load librfx.so (building it in-tree first if it is missing/stale and hipcc exists)."""
    global _lib
    if _lib is not None:
        return _lib
    path = _build.LIB
    if build_if_missing:
        try:
            _build.build()
        except Exception as e:  # no hipcc on this host: only an existing library will do
            if not os.path.exists(path):
                raise RfxError(f"librfx.so missing and cannot be built: {e}") from e
    if not os.path.exists(path):
        raise RfxError(f"librfx.so not found at {path}: the HIP renderer is required (no CPU fallback)")
    L = C.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.rfx_abi_version() != RFX_ABI_VERSION:
        raise RfxError("librfx.so ABI version mismatch")
    _lib = L
    return L


def lib_sha256(path: str = None) -> str:
    """SHA-256 of the library file (keys the PMC records of profiles/pmc to the build they measured)."""
    import hashlib
    with open(path or _build.LIB, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def device_sha256(path: str = None) -> str:
    """SHA-256 of the library's device code (its .hip_fatbin ELF section: every kernel's code object).  Host-only
    changes leave it alone (the build is deterministic), so it keys the PMC records of profiles/pmc to the
    kernels they measured; None if the section is absent."""
    import hashlib
    import struct
    with open(path or _build.LIB, "rb") as f:
        b = f.read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    for name_off, _, _, _, off, size, *_ in secs:
        if b[names + name_off:b.index(b"\0", names + name_off)] == b".hip_fatbin":
            return hashlib.sha256(b[off:off + size]).hexdigest()
    return None


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = load().rfx_last_error().decode(errors="replace")
        raise RfxError(f"{what or 'rfx call'} failed ({rc}): {msg}")
    return rc


def fptr(a):
    return a.ctypes.data_as(_fp)


def u32ptr(a):
    return a.ctypes.data_as(_u32p)


def u64ptr(a):
    return a.ctypes.data_as(_u64p)


def farr(v, n=None):
    v = list(v)
    if n is not None and len(v) != n:
        raise ValueError(f"expected {n} floats, got {len(v)}")
    return (C.c_float * len(v))(*v)
