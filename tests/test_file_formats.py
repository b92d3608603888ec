"""File formats against the reference's own bytes (tests/golden/file_*.npz, tools/gen_golden.py).

* file_save: the bytes Texture::saveToBMPFile / saveToTGAFile wrote for a 7x5 ARGB image
  (Texture.cpp:110-173, image_headers.h) -- rfx_bmp_save / rfx_tga_save must write the same bytes;
  saveToFile(".png") returns false (Texture.cpp:195-207).
* file_load: what Texture::loadFromFile (Texture.cpp:34-108, 175-189) made of hand-made TGA files -- 24/32
  bpp, an id field, colour-map fields, the origin bit, a > 32768-pixel image (the reader's buffer refills),
  trailing bytes, truncated pixels and header, other image types and depths, an empty file, a wrong
  extension and a zero width -- rfx_scene_add_texture_file / rfx_tga_load must agree on success, size and
  every texel.
No GPU: these are the host side of the C-ABI.
"""
import ctypes as C
import os

import numpy as np

from helpers import GOLDEN
from reflaxman_amd import _lib


def test_save_bytes_match_reference(tmp_path):
    g = np.load(os.path.join(GOLDEN, "file_save.npz"))
    L = _lib.load()
    img = np.ascontiguousarray(g["argb"], np.uint32)
    h, w = img.shape
    assert g["ok"].tolist() == [1, 1, 0]
    for ext, fn in (("bmp", L.rfx_bmp_save), ("tga", L.rfx_tga_save)):
        p = str(tmp_path / f"x.{ext}")
        assert fn(p.encode(), w, h, _lib.u32ptr(img)) == 0
        data = np.fromfile(p, np.uint8)
        assert data.tobytes() == g[ext].tobytes(), ext


def test_tga_loads_match_reference(tmp_path):
    g = np.load(os.path.join(GOLDEN, "file_load.npz"))
    L = _lib.load()
    names = [str(n) for n in g["names"]]
    assert len(names) >= 12
    for i, name in enumerate(names):
        p = str(tmp_path / name)
        g[f"in{i}"].tofile(p)
        ref = g[f"out{i}"]
        ok, rw, rh = int(ref[0]), int(ref[1]), int(ref[2])
        # Scene::addTexture(fileName) -> Texture(fileName) -> loadFromFile (extension check, then TGA)
        s = L.rfx_scene_create(0, 0, 0, 0)
        loaded = C.c_int(-1)
        assert L.rfx_scene_add_texture_file(s, p.encode(), C.byref(loaded)) == 0
        L.rfx_scene_destroy(s)
        assert loaded.value == ok, name
        if not name.endswith(".tga"):
            continue
        w, h = C.c_uint32(), C.c_uint32()
        rc = L.rfx_tga_load(p.encode(), C.byref(w), C.byref(h), None, 0)
        assert (rc == 0) == bool(ok), name
        if not ok:
            continue
        assert (w.value, h.value) == (rw, rh), name
        buf = np.zeros(max(1, rw * rh), np.uint32)
        assert L.rfx_tga_load(p.encode(), C.byref(w), C.byref(h), _lib.u32ptr(buf), buf.size) == 0
        assert np.array_equal(buf[: rw * rh], ref[3:]), name
