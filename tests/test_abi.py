"""C-ABI checks that need no GPU: the library loads, exports every symbol
include/rfx.h declares, and its host-side precompute matches the reference."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from helpers import GOLDEN
from reflaxman_amd import _lib, scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "rfx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rfx_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = _lib.load()
    names = declared_symbols()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_no_gpu_is_a_loud_error():
    """Without a device the renderer refuses (there is no CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = _lib.load()
    h = C.c_void_p()
    assert L.rfx_renderer_create(C.byref(h), 0) == -6  # RFX_ERR_NODEV
    with pytest.raises(_lib.RfxError):
        from reflaxman_amd.render import Render
        Render()


def test_camera_view_matches_reference_kat():
    g = np.load(os.path.join(GOLDEN, "kat_camera.npz"))
    L = _lib.load()
    out = np.zeros((g["inp"].shape[0], 9), np.float32)
    for i, r in enumerate(g["inp"]):
        L.rfx_camera_view(_lib.farr(r[0:3]), _lib.farr(r[3:6]), out[i].ctypes.data_as(C.POINTER(C.c_float)))
    assert out.tobytes() == g["out"].tobytes()


def test_argb_matches_reference_kat():
    g = np.load(os.path.join(GOLDEN, "kat_argb.npz"))
    inp = np.ascontiguousarray(g["inp"], np.float32)
    out = np.zeros(inp.shape[0], np.uint32)
    _lib.load().rfx_argb_from_rgb(_lib.fptr(inp), inp.shape[0], _lib.u32ptr(out))
    assert np.array_equal(out, g["out"])


def test_tga_roundtrip_and_bmp_layout(tmp_path):
    L = _lib.load()
    tex = scenes.synth_texture("t", 37, 21, 99).argb
    p = str(tmp_path / "a.tga")
    scenes.write_tga(p, tex, bpp=24)
    w, h = C.c_uint32(), C.c_uint32()
    assert L.rfx_tga_load(p.encode(), C.byref(w), C.byref(h), None, 0) == 0 and (w.value, h.value) == (37, 21)
    buf = np.zeros((21, 37), np.uint32)
    assert L.rfx_tga_load(p.encode(), C.byref(w), C.byref(h), _lib.u32ptr(buf), buf.size) == 0
    assert np.array_equal(buf, (tex & 0x00FFFFFF) | 0xFF000000)  # 24 bpp -> alpha 0xFF (Texture.cpp:87)
    assert np.array_equal(scenes.read_tga(p), buf)
    # 32-bpp write -> read back
    q = str(tmp_path / "b.tga")
    assert L.rfx_tga_save(q.encode(), 37, 21, _lib.u32ptr(np.ascontiguousarray(tex))) == 0
    assert np.array_equal(scenes.read_tga(q), tex)
    # BMP: 54-byte header, 32 bpp, rows as stored (bottom-up, Texture.cpp:139-173)
    b = str(tmp_path / "c.bmp")
    assert L.rfx_bmp_save(b.encode(), 37, 21, _lib.u32ptr(np.ascontiguousarray(tex))) == 0
    data = open(b, "rb").read()
    assert data[:2] == b"BM" and len(data) == 54 + 37 * 21 * 4
    assert np.array_equal(np.frombuffer(data[54:], np.uint32).reshape(21, 37), tex)
    assert L.rfx_tga_load(b"/nonexistent/x.tga", C.byref(w), C.byref(h), None, 0) == -4


def test_scene_builder_counts_and_errors():
    from reflaxman_amd.render import Color, Material, Scene, Vector3, build_scene
    s, cam = build_scene(scenes.synth16_scene(tex_size=8))
    assert s.counts() == (16, 4, 1, 2)
    with pytest.raises(ValueError):
        Material(7)
    L = _lib.load()
    assert L.rfx_triangle_set_texture(s._h, 0, 0, _lib.farr([0] * 6)) == -1  # object 0 is a sphere
    assert L.rfx_scene_add_texture_file(s._h, b"/nonexistent/x.tga", None) >= 0  # failed load -> checker texture


def test_strip_partition_covers_every_row_once():
    L = _lib.load()
    for H in (1, 7, 64, 123, 2160, 4320):
        for nr in (1, 2, 3, 4, 8):
            for rb in (1, 5, 8, 16):
                seen = []
                for rank in range(nr):
                    rows = L.rfx_strip_rows(H, rb, rank, nr)
                    seen += [L.rfx_strip_row_to_y(i, rb, rank, nr) for i in range(rows)]
                assert sorted(seen) == list(range(H)), (H, nr, rb)
