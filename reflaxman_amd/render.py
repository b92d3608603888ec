"""Python mirror of the reference's Render / Scene / Camera / Material API.

Same names, argument meaning and error behaviour as the reference's C++
classes (src/common/Render.h:7-42, Scene.h:28-40, Camera.h:30-62,
Material.h:5-19, OmniLight.h, Color.h, Vector3.h, Texture.h), implemented over
the C-ABI of librfx.so (include/rfx.h).  Every trace runs in the HIP kernels;
there is no CPU path.

Drop-in semantics (Render.cpp:57-226):
  * ``setImageSize`` zero-fills the float framebuffer, resets the cursor and
    ``additiveCounter``;
  * ``renderBegin`` snapshots the camera and bumps/clears ``additiveCounter``;
  * ``renderNext(pixels)`` renders exactly the raster span the reference's
    cursor would cover -- on the GPU, one launch per call -- and returns
    ``inProgress``.  Chunked callers (Pulse.cpp:102-209) therefore get the
    reference's image for any chunk pattern;
  * ``renderAll`` keeps the reference's behaviour (renders ``imageHeight``
    *pixels*, Render.cpp:217-221);
  * ``imagePixel`` divides by ``additiveCounter`` when it is > 1, ``copyImage``
    does not (Render.cpp:82-114).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import _lib
from ._lib import DIELECTRIC, METAL, check, farr

DEFAULT_SPHERE_SEED = 1350490027  # glibc rand() #12: Vector3.cpp's stream in the survey's link order
DEFAULT_JITTER_SEED = 424238335   # glibc rand() #6:  Render.cpp's stream in the same link order


class Vector3:
    __slots__ = ("x", "y", "z")

    def __init__(self, x=0.0, y=0.0, z=0.0):
        self.x, self.y, self.z = float(x), float(y), float(z)

    def __iter__(self):
        return iter((self.x, self.y, self.z))

    def __repr__(self):
        return f"Vector3({self.x}, {self.y}, {self.z})"


class Color:
    __slots__ = ("r", "g", "b")

    def __init__(self, r=0.0, g=0.0, b=0.0):
        self.r, self.g, self.b = float(r), float(g), float(b)

    def __iter__(self):
        return iter((self.r, self.g, self.b))

    def argb(self) -> int:
        """Color::argb (Color.cpp:114-117)."""
        out = (C.c_uint32 * 1)()
        _lib.load().rfx_argb_from_rgb(farr(self), 1, out)
        return int(out[0])

    def __repr__(self):
        return f"Color({self.r}, {self.g}, {self.b})"


class Material:
    """Material(type, color, reflectivity, transparency) -- Material.cpp:8-14 (clamping happens in the library)."""
    mtMetal, mtDielectric = METAL, DIELECTRIC

    def __init__(self, type=METAL, color: Color = Color(1, 1, 1), reflectivity=0.0, transparency=0.0):
        if type not in (METAL, DIELECTRIC):
            raise ValueError("Material type must be Material.mtMetal or Material.mtDielectric")
        self.type = type
        self.color = Color(*color)
        self.reflectivity = float(reflectivity)
        self.transparency = float(transparency)


class Camera:
    """Camera(eye, at, fov): the rendering-relevant part (Camera.cpp:24-56).  ``view`` is row-major _11.._33."""

    def __init__(self, eye=Vector3(), at=Vector3(0, 0, 1), fov=1.0):
        self.eye = Vector3(*eye)
        self.fov = float(fov)
        view = (C.c_float * 9)()
        _lib.load().rfx_camera_view(farr(self.eye), farr(Vector3(*at)), view)
        self.view = [float(v) for v in view]


class Texture:
    """Handle of a scene texture (Scene::addTexture's returned Texture*)."""

    def __init__(self, scene: "Scene", index: int, loaded: bool):
        self.scene, self.index, self.loaded = scene, index, loaded


class Triangle:
    """Handle of a scene triangle (Scene::addTriangle's returned Triangle*)."""

    def __init__(self, scene: "Scene", obj: int):
        self.scene, self.obj = scene, obj

    def setTexture(self, texture: Optional[Texture], u1, v1, u2, v2, u3, v3):  # Triangle.cpp:110-120
        if texture is None:
            raise ValueError("setTexture needs a texture from Scene.addTexture")
        check(_lib.load().rfx_triangle_set_texture(self.scene._h, self.obj, texture.index, farr((u1, v1, u2, v2, u3, v3))),
              "Triangle.setTexture")
        self.scene._version += 1


class Sphere:
    def __init__(self, scene: "Scene", obj: int):
        self.scene, self.obj = scene, obj


class Plane:
    """Handle of a scene plane (Scene.addPlane, the extension of Scene::add* to Plane.h's primitive)."""

    def __init__(self, scene: "Scene", obj: int):
        self.scene, self.obj = scene, obj


class OmniLight:
    def __init__(self, scene: "Scene", index: int):
        self.scene, self.index = scene, index


class Scene:
    """Scene(diffLightColor, diffLightPower) -- Scene.cpp:10-71."""

    def __init__(self, diffLightColor: Color = Color(0, 0, 0), diffLightPower: float = 0.0):
        L = _lib.load()
        self._h = C.c_void_p(L.rfx_scene_create(*Color(*diffLightColor), float(diffLightPower)))
        if not self._h:
            raise _lib.RfxError("rfx_scene_create failed")
        self._version = 0
        self._keep = []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib._lib is not None:
            _lib._lib.rfx_scene_destroy(h)
            self._h = None

    def addSphere(self, center: Vector3, radius: float, material: Material) -> Sphere:
        obj = check(_lib.load().rfx_scene_add_sphere(self._h, farr(Vector3(*center)), float(radius), material.type,
                                                     farr(material.color), material.reflectivity, material.transparency),
                    "Scene.addSphere")
        self._version += 1
        return Sphere(self, obj)

    def addTriangle(self, v1: Vector3, v2: Vector3, v3: Vector3, material: Material) -> Triangle:
        obj = check(_lib.load().rfx_scene_add_triangle(self._h, farr(Vector3(*v1)), farr(Vector3(*v2)), farr(Vector3(*v3)),
                                                       material.type, farr(material.color), material.reflectivity,
                                                       material.transparency), "Scene.addTriangle")
        self._version += 1
        return Triangle(self, obj)

    def addPlane(self, pos: Vector3, norm: Vector3, material: Material) -> Plane:
        """Plane(pos, norm, material) (Plane.cpp:9-14) as a scene object, traced by Plane::trace (Plane.cpp:36-73)."""
        obj = check(_lib.load().rfx_scene_add_plane(self._h, farr(Vector3(*pos)), farr(Vector3(*norm)), material.type,
                                                    farr(material.color), material.reflectivity, material.transparency),
                    "Scene.addPlane")
        self._version += 1
        return Plane(self, obj)

    def addLight(self, origin: Vector3, radius: float, color: Color, power: float) -> OmniLight:
        idx = check(_lib.load().rfx_scene_add_light(self._h, farr(Vector3(*origin)), float(radius), farr(Color(*color)),
                                                    float(power)), "Scene.addLight")
        self._version += 1
        return OmniLight(self, idx)

    def addTexture(self, fileName: str) -> Texture:
        """Scene::addTexture(fileName): TGA; a failed load gives the checker texture, like the reference."""
        loaded = C.c_int(0)
        idx = check(_lib.load().rfx_scene_add_texture_file(self._h, os.fsencode(fileName), C.byref(loaded)),
                    "Scene.addTexture")
        self._version += 1
        return Texture(self, idx, bool(loaded.value))

    def addTextureArgb(self, argb: Optional[np.ndarray]) -> Texture:
        """Texture from an (h, w) uint32 ARGB array; None = empty (checker)."""
        L = _lib.load()
        if argb is None:
            idx = check(L.rfx_scene_add_texture_argb(self._h, 0, 0, None), "Scene.addTextureArgb")
        else:
            a = np.ascontiguousarray(argb, dtype=np.uint32)
            idx = check(L.rfx_scene_add_texture_argb(self._h, a.shape[1], a.shape[0], _lib.u32ptr(a)), "Scene.addTextureArgb")
        self._version += 1
        return Texture(self, idx, argb is not None)

    def setSkyboxTexture(self, fileName: str) -> bool:
        ok = check(_lib.load().rfx_scene_set_skybox_file(self._h, os.fsencode(fileName)), "Scene.setSkyboxTexture")
        self._version += 1
        return bool(ok)

    def setSkyboxTextureArgb(self, argb: Optional[np.ndarray]) -> bool:
        L = _lib.load()
        if argb is None:
            ok = check(L.rfx_scene_set_skybox_argb(self._h, 0, 0, None), "Scene.setSkyboxTextureArgb")
        else:
            a = np.ascontiguousarray(argb, dtype=np.uint32)
            ok = check(L.rfx_scene_set_skybox_argb(self._h, a.shape[1], a.shape[0], _lib.u32ptr(a)), "Scene.setSkyboxTextureArgb")
        self._version += 1
        return bool(ok)

    def counts(self):
        v = [C.c_int() for _ in range(4)]
        check(_lib.load().rfx_scene_counts(self._h, *[C.byref(x) for x in v]), "Scene.counts")
        return tuple(x.value for x in v)


def build_scene(desc, texture_dir: Optional[str] = None) -> tuple:
    """Replay a :class:`reflaxman_amd.scenes.SceneDesc` through the Scene API; returns (Scene, Camera).

    texture_dir: write the textures as TGA files there (SceneDesc.write) and load them through
    Scene.addTexture / setSkyboxTexture (the library's TGA reader), as the reference's loadScene does."""
    d = desc.diffuse
    s = Scene(Color(d[0], d[1], d[2]), d[3])
    files = {}
    if texture_dir is not None:
        path = desc.write(texture_dir)
        for line in open(path):
            parts = line.split()
            if parts and parts[0] in ("skybox", "texture"):
                files.setdefault(parts[0], []).append(
                    None if parts[1] == "-" else os.path.join(texture_dir, parts[1]))
    if desc.skybox is not None:
        if texture_dir is not None:
            s.setSkyboxTexture(files["skybox"][0] or "/nonexistent/absent.tga")
        else:
            s.setSkyboxTextureArgb(desc.skybox.argb)
    for (o, r, c, p) in desc.lights:
        s.addLight(Vector3(*o), r, Color(*c), p)
    if texture_dir is not None:
        texs = [s.addTexture(f or "/nonexistent/absent.tga") for f in files.get("texture", [])]
    else:
        texs = [s.addTextureArgb(t.argb) for t in desc.textures]
    handles = []
    for ob in desc.objects:
        mt, rgb, refl, tr = ob[-1]
        m = Material(mt, Color(*rgb), refl, tr)
        if ob[0] == "sphere":
            handles.append(s.addSphere(Vector3(*ob[1]), ob[2], m))
        elif ob[0] == "plane":
            handles.append(s.addPlane(Vector3(*ob[1]), Vector3(*ob[2]), m))
        else:
            handles.append(s.addTriangle(Vector3(*ob[1]), Vector3(*ob[2]), Vector3(*ob[3]), m))
    for (oi, ti, uv) in desc.settex:
        handles[oi].setTexture(texs[ti], *uv)
    eye, at, fov = desc.camera
    return s, Camera(Vector3(*eye), Vector3(*at), fov)


class Renderer:
    """Thin owner of an rfx_renderer (device, stream, uploaded scene, RNG streams)."""

    def __init__(self, device: int = 0, sphere_seed: int = DEFAULT_SPHERE_SEED, jitter_seed: int = DEFAULT_JITTER_SEED):
        L = _lib.load()
        h = C.c_void_p()
        check(L.rfx_renderer_create(C.byref(h), int(device)), "rfx_renderer_create")
        self._h = h
        self.device = device
        self._scene_key = None
        self.set_rng(sphere_seed, jitter_seed)

    def close(self):
        if getattr(self, "_h", None) and _lib._lib is not None:
            _lib._lib.rfx_renderer_destroy(self._h)
            self._h = None

    __del__ = close

    def set_scene(self, scene: Scene):
        key = (id(scene), scene._version)
        if key != self._scene_key:
            check(_lib.load().rfx_renderer_set_scene(self._h, scene._h), "rfx_renderer_set_scene")
            self._scene_key = key
            self._scene_ref = scene

    def set_rng(self, sphere_seed: int, jitter_seed: int):
        check(_lib.load().rfx_renderer_set_rng(self._h, sphere_seed & 0xFFFFFFFF, jitter_seed & 0xFFFFFFFF), "set_rng")

    def get_rng(self):
        s, j = C.c_uint32(), C.c_uint32()
        check(_lib.load().rfx_renderer_get_rng(self._h, C.byref(s), C.byref(j)), "get_rng")
        return s.value, j.value

    def set_stream(self, stream_ptr: int):
        check(_lib.load().rfx_renderer_set_stream(self._h, C.c_void_p(stream_ptr)), "set_stream")

    def render_frame(self, frame: _lib.Frame, d_rgb: int, d_argb: int = 0, d_counters: int = 0, stream: int = 0):
        """Enqueue one frame into caller-owned device buffers (device pointers as ints)."""
        check(_lib.load().rfx_render_frame(self._h, C.byref(frame), C.c_void_p(d_rgb), C.c_void_p(d_argb or None),
                                           C.c_void_p(d_counters or None), C.c_void_p(stream or None)), "rfx_render_frame")

    def synchronize(self):
        check(_lib.load().rfx_synchronize(self._h), "rfx_synchronize")

    def set_tile_order(self, mode: int):
        """Trace-launch schedule (rfx.h rfx_renderer_set_tile_order): 1 longest-tile-first (8x8 wave tiles)
        from earlier launches' tile costs on large launches (default), 3 on every launch, 0 raster order,
        2 raster order with cost recording.  No pixel changes."""
        check(_lib.load().rfx_renderer_set_tile_order(self._h, int(mode)), "set_tile_order")

    def set_prim_masks(self, mode: int):
        """Primary-bundle cull masks of small-scene plain and SSAA frames (rfx.h rfx_renderer_set_prim_masks): 1 built
        when a view repeats (default; sampleNum > 8: every view), 2 before every launch, 0 off.  No pixel changes.  Any
        call forgets the views seen so far."""
        check(_lib.load().rfx_renderer_set_prim_masks(self._h, int(mode)), "set_prim_masks")

    def set_regroup(self, park_after: int):
        """Ray regrouping (rfx.h rfx_renderer_set_regroup): -1 default (large scenes, after 2 segments), 0 off,
        n >= 1 park traces alive after n segments for the packed bounce kernel.  No pixel changes."""
        check(_lib.load().rfx_renderer_set_regroup(self._h, int(park_after)), "set_regroup")

    def set_regroup_sort(self, on: bool):
        """Regrouped frames (rfx.h rfx_renderer_set_regroup_sort): the bounce kernel takes the parked traces sorted
        by direction octant and origin cell, or in park order (default).  No pixel changes."""
        check(_lib.load().rfx_renderer_set_regroup_sort(self._h, int(bool(on))), "set_regroup_sort")

    def set_launch_traces(self, max_traces: int):
        """The most traces one launch takes (rfx.h rfx_renderer_set_launch_traces; 0 = the default 2^30): larger spans
        render as consecutive launches.  No pixel changes."""
        check(_lib.load().rfx_renderer_set_launch_traces(self._h, int(max_traces)), "set_launch_traces")

    def bounce_form(self) -> int:
        """The last trace launch's bounce kernel (rfx.h rfx_renderer_bounce_form): 0 none, 1 global-memory BVH, 2 the
        LDS-staged BVH."""
        return _lib.load().rfx_renderer_bounce_form(self._h)

    def set_timing(self, enable):
        """HIP-event timing of the frames (rfx.h rfx_renderer_set_timing): True / 1 every frame, n > 1 every n-th
        frame, False / 0 off."""
        check(_lib.load().rfx_renderer_set_timing(self._h, int(enable)), "set_timing")

    def get_timing(self):
        """(prepass_ms, trace_ms, frames) summed over the frames since the last call (HIP events)."""
        a, b, n = C.c_double(), C.c_double(), C.c_uint64()
        check(_lib.load().rfx_renderer_get_timing(self._h, C.byref(a), C.byref(b), C.byref(n)), "get_timing")
        return a.value, b.value, n.value

    # device known-answer entry points (rfx.h rfx_kat_*), on the uploaded scene
    def kat_objects(self, rays: np.ndarray, objects: np.ndarray) -> np.ndarray:
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        objs = np.ascontiguousarray(objects, np.int32)
        out = np.zeros((rays.shape[0], 15), np.float32)
        check(_lib.load().rfx_kat_objects(self._h, _lib.fptr(rays), objs.ctypes.data_as(C.POINTER(C.c_int32)),
                                          rays.shape[0], _lib.fptr(out)), "rfx_kat_objects")
        return out

    def kat_texels(self, texture: int, inp: np.ndarray) -> np.ndarray:
        inp = np.ascontiguousarray(inp, np.float32)
        out = np.zeros((inp.shape[0], 3), np.float32)
        check(_lib.load().rfx_kat_texels(self._h, int(texture), _lib.fptr(inp), inp.shape[0], _lib.fptr(out)),
              "rfx_kat_texels")
        return out

    def kat_powf(self, xy: np.ndarray) -> np.ndarray:
        xy = np.ascontiguousarray(xy, np.float32)
        out = np.zeros(xy.shape[0], np.float32)
        check(_lib.load().rfx_kat_powf(self._h, _lib.fptr(xy), xy.shape[0], _lib.fptr(out)), "rfx_kat_powf")
        return out

    def kat_powf_cube(self):
        """(mismatches, glibc-path inputs) of the Fresnel cube form vs glibc's algorithm over every float in [0, 1]."""
        counts = (C.c_uint64 * 2)()
        check(_lib.load().rfx_kat_powf_cube(self._h, counts), "rfx_kat_powf_cube")
        return int(counts[0]), int(counts[1])

    def kat_argb(self, rgb: np.ndarray) -> np.ndarray:
        rgb = np.ascontiguousarray(rgb, np.float32)
        out = np.zeros(rgb.shape[0], np.uint32)
        check(_lib.load().rfx_kat_argb(self._h, _lib.fptr(rgb), rgb.shape[0], _lib.u32ptr(out)), "rfx_kat_argb")
        return out

    def rand_dirs(self, seed: int, n: int):
        out = np.zeros((n, 3), np.float32)
        after = C.c_uint32()
        check(_lib.load().rfx_rand_dirs(self._h, seed, n, _lib.fptr(out), C.byref(after)), "rfx_rand_dirs")
        return out, after.value


def make_frame(camera: Camera, W: int, H: int, reflect_num: int, sample_num: int = 1, additive: bool = False,
               additive_counter: int = 0, row_block: int = 0, rank: int = 0, nranks: int = 1,
               pixel_begin: int = 0, pixel_end: int = 0) -> _lib.Frame:
    f = _lib.Frame()
    f.eye[:] = list(camera.eye)
    f.view[:] = list(camera.view)
    f.fov = camera.fov
    f.width, f.height = W, H
    f.reflect_num, f.sample_num = reflect_num, sample_num
    f.additive, f.additive_counter = int(bool(additive)), additive_counter
    f.row_block, f.rank, f.nranks = row_block, rank, nranks
    f.pixel_begin, f.pixel_end = pixel_begin, pixel_end
    return f


class Render:
    """Render (Render.h:7-42) over the GPU renderer."""

    def __init__(self, exePath: str = "", device: int = 0, sphere_seed: int = DEFAULT_SPHERE_SEED,
                 jitter_seed: int = DEFAULT_JITTER_SEED, load_default_scene: bool = True):
        self._r = Renderer(device, sphere_seed, jitter_seed)
        self.imageWidth = 0
        self.imageHeight = 0
        self.additiveCounter = 0
        self.inProgress = False
        self._curx = 0
        self._cury = 0
        self._d_img = None
        self._cap = 0
        self._host = None
        self._host_valid = False
        self.camera = Camera()
        self.scene = Scene()
        self._refl = 0
        self._ss = 0
        self._additive = False
        if load_default_scene:
            self.loadScene(exePath)

    def loadScene(self, exePath: str):
        """Render::loadScene (Render.cpp:25-55)."""
        from . import scenes
        sky = os.path.join(exePath, "./textures/skybox.tga")
        plane = os.path.join(exePath, "./textures/himiya.tga")
        self.camera = Camera(Vector3(*scenes.DEFAULT_CAMERA[0]), Vector3(*scenes.DEFAULT_CAMERA[1]), scenes.DEFAULT_CAMERA[2])
        self.scene = Scene(Color(0.95, 0.95, 1.0), 0.15)
        self.scene.setSkyboxTexture(sky)
        self.scene.addLight(Vector3(11.8e9, 4.26e9, 3.08e9), 3.48e8, Color(1.0, 1.0, 0.95), 0.85)
        for (c, r, mt, rgb, refl) in [
            ((-1.25, 1.5, -0.25), 1.5, METAL, (1.0, 1.0, 1.0), 1.0), ((0.15, 1.0, 1.75), 1.0, METAL, (1.0, 1.0, 1.0), 0.95),
            ((-3.0, 0.6, -3.0), 0.6, DIELECTRIC, (1.0, 1.0, 1.0), 0.0), ((-0.5, 0.5, -2.5), 0.5, DIELECTRIC, (0.5, 1.0, 0.15), 0.75),
            ((1.0, 0.4, -1.5), 0.4, DIELECTRIC, (0.0, 0.5, 1.0), 1.0), ((1.8, 0.4, 0.1), 0.4, METAL, (1.0, 0.65, 0.45), 1.0),
            ((1.7, 0.5, 1.9), 0.5, METAL, (1.0, 0.90, 0.60), 0.75), ((0.6, 0.6, 4.2), 0.6, METAL, (0.9, 0.9, 0.9), 0.0)]:
            self.scene.addSphere(Vector3(*c), r, Material(mt, Color(*rgb), refl, 0.0))
        tex = self.scene.addTexture(plane)
        tr1 = self.scene.addTriangle(Vector3(-14.0, 0.0, -10.0), Vector3(-14.0, 0.0, 10.0), Vector3(14.0, 0.0, -10.0),
                                     Material(DIELECTRIC, Color(1.0, 1.0, 1.0), 0.95, 0.0))
        tr1.setTexture(tex, 0.0, 0.0, 0.0, 1.0, 1.0, 0.0)
        tr2 = self.scene.addTriangle(Vector3(-14.0, 0.0, 10.0), Vector3(14.0, 0.0, 10.0), Vector3(14.0, 0.0, -10.0),
                                     Material(DIELECTRIC, Color(1.0, 1.0, 1.0), 0.95, 0.0))
        tr2.setTexture(tex, 0.0, 1.0, 1.0, 1.0, 1.0, 0.0)

    # -- image buffer ------------------------------------------------------
    def setImageSize(self, width: int, height: int):                      # Render.cpp:57-80
        if width <= 0 or height <= 0:
            return
        L = _lib.load()
        n = width * height * 3 * 4
        if n > self._cap:
            if self._d_img:
                check(L.rfx_device_free(self._r._h, self._d_img), "device_free")
                self._d_img = None
            p = C.c_void_p()
            check(L.rfx_device_alloc(self._r._h, n, C.byref(p)), "device_alloc")
            self._d_img, self._cap = p, n
        zeros = np.zeros(width * height * 3, np.float32)
        check(L.rfx_memcpy_h2d(self._r._h, self._d_img, zeros.ctypes.data_as(C.c_void_p), n), "memcpy_h2d")
        self.imageWidth, self.imageHeight = width, height
        self.additiveCounter = 0
        self.inProgress = False
        self._curx = self._cury = 0
        self._host_valid = False

    def _image(self) -> np.ndarray:
        if not self._host_valid:
            n = self.imageWidth * self.imageHeight
            self._host = np.empty((self.imageHeight, self.imageWidth, 3), np.float32)
            check(_lib.load().rfx_memcpy_d2h(self._r._h, self._host.ctypes.data_as(C.c_void_p), self._d_img, n * 12), "memcpy_d2h")
            self._host_valid = True
        return self._host

    @property
    def image(self) -> np.ndarray:
        """The float framebuffer (std::vector<Color> image, Render.h:10), row 0 = bottom."""
        return self._image()

    def imagePixel(self, x: int, y: int) -> Color:                       # Render.cpp:103-114
        if x < 0 or y < 0:
            return Color(0, 0, 0)
        c = self._image()[y, x]
        if self.additiveCounter > 1:
            k = np.float32(self.additiveCounter)
            return Color(*(c / k).astype(np.float32))
        return Color(*c)

    def imagePixels(self) -> np.ndarray:
        """imagePixel for every pixel at once."""
        img = self._image()
        if self.additiveCounter > 1:
            return (img / np.float32(self.additiveCounter)).astype(np.float32)
        return img.copy()

    def copyImage(self) -> np.ndarray:                                   # Render.cpp:82-101
        """ARGB (h, w) uint32 of the stored (not averaged) image, as Render::copyImage writes a Texture."""
        img = np.ascontiguousarray(self._image())
        out = np.empty((self.imageHeight, self.imageWidth), np.uint32)
        _lib.load().rfx_argb_from_rgb(_lib.fptr(img), img.shape[0] * img.shape[1], _lib.u32ptr(out))
        return out

    # -- rendering ---------------------------------------------------------
    def renderBegin(self, reflectNum: int, sampleNum: int, additive: bool):  # Render.cpp:116-134
        if reflectNum <= 0 or sampleNum == 0:
            raise ValueError("renderBegin: reflectNum > 0 and sampleNum != 0 required (reference asserts)")
        self._refl, self._ss, self._additive = reflectNum, sampleNum, bool(additive)
        self.inProgress = True
        self._curx = self._cury = 0
        self._view = list(self.camera.view)
        self._eye = Vector3(*self.camera.eye)
        self.additiveCounter = self.additiveCounter + 1 if additive else 0

    def renderNext(self, pixels: int) -> bool:                              # Render.cpp:136-215
        W, H = self.imageWidth, self.imageHeight
        if not pixels or not self.inProgress or self._curx >= W or self._cury >= H:
            return False
        p0 = self._cury * W + self._curx
        p1 = min(p0 + pixels, W * H)
        cam = Camera.__new__(Camera)
        cam.eye, cam.view, cam.fov = self._eye, self._view, self.camera.fov
        self._r.set_scene(self.scene)
        f = make_frame(cam, W, H, self._refl, self._ss, self._additive, self.additiveCounter,
                       pixel_begin=p0, pixel_end=p1)
        self._r.render_frame(f, self._d_img.value)
        self._host_valid = False
        self._curx, self._cury = p1 % W, p1 // W
        if p1 == W * H:
            self._curx, self._cury = 0, H
            self.inProgress = False
        return self.inProgress

    def renderAll(self, reflectNum: int, sampleNum: int, additive: bool):   # Render.cpp:217-221 (sic)
        self.renderBegin(reflectNum, sampleNum, additive)
        self.renderNext(self.imageHeight)

    def getRenderProgress(self) -> float:                                   # Render.cpp:223-226
        W, H = self.imageWidth, self.imageHeight
        return float(np.float32(self._curx + self._cury * W) * np.float32(100.0) / np.float32(W) / np.float32(H))

    def getRng(self):
        return self._r.get_rng()

    def synchronize(self):
        self._r.synchronize()

    def close(self):
        L = _lib._lib
        if getattr(self, "_d_img", None) and L is not None and self._r._h:
            L.rfx_device_free(self._r._h, self._d_img)
            self._d_img = None
        self._r.close()
