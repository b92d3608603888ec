"""Scene descriptions for the parity cases and the benchmark workloads.

A scene is an *ordered list of reference API calls* -- exactly the calls
``Render::loadScene`` makes (reference src/common/Render.cpp:25-55):
``Scene(diffColor, diffPower)``, ``setSkyboxTexture``, ``addLight``,
``addSphere``, ``addTexture``, ``addTriangle`` + ``Triangle::setTexture``, and
``Camera(eye, at, fov)``.  Order matters for parity: object order decides
closest-hit ties (Scene.cpp:98, first inserted wins) and ``envColor``
accumulates in ``addLight`` order (Scene.cpp:55).

The same list is written to a plain-text ``.scene`` file (floats as C99 hex
literals, bit-exact) that the oracle harness replays through the reference's
own API, and replayed by :func:`reflaxman_amd.render.build_scene` through our
C-ABI.  Textures are ARGB ``uint32`` arrays (texel row = file row, the TGA
origin bit is ignored as in Texture.cpp:34-108) or ``None`` for a failed load,
which the reference turns into its procedural 50x50 grey checker
(Texture.cpp:242-243).

Workloads (SURVEY.md §8 / BASELINE.json configs):
  ``default``     -- C1/C2: Render::loadScene verbatim, textures absent.
  ``synth16``     -- C3/C4: 16 spheres (8 default + 8 LCG) + ground quad + back
                     wall quad (4 textured triangles) + the default sun.
  ``stress4096``  -- C5: 4096 LCG spheres + ground quad.
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

METAL, DIELECTRIC = 0, 1

F32 = np.float32


def f32(x) -> float:
    """Round a Python float to the nearest float32 (as the reference's float literals are)."""
    return float(np.float32(x))


@dataclass
class Texture:
    name: str
    argb: Optional[np.ndarray]  # (h, w) uint32 or None -> empty texture (checker)

    @property
    def width(self) -> int:
        return 0 if self.argb is None else int(self.argb.shape[1])

    @property
    def height(self) -> int:
        return 0 if self.argb is None else int(self.argb.shape[0])


@dataclass
class SceneDesc:
    name: str
    diffuse: Tuple[float, float, float, float]          # Scene(Color(r,g,b), power)
    camera: Tuple[Tuple[float, float, float], Tuple[float, float, float], float]
    skybox: Optional[Texture] = None                      # setSkyboxTexture; None == absent
    textures: List[Texture] = field(default_factory=list)  # addTexture order
    lights: List[tuple] = field(default_factory=list)      # (origin3, radius, rgb3, power)
    objects: List[tuple] = field(default_factory=list)     # ('sphere', c3, r, mat) | ('triangle', v0, v1, v2, mat)
                                                           # | ('plane', pos3, norm3, mat)
    settex: List[tuple] = field(default_factory=list)      # (object_index, texture_index, uv6)

    # ---- builders (mirroring the reference calls) ----
    def add_light(self, origin, radius, rgb, power):
        self.lights.append((tuple(map(f32, origin)), f32(radius), tuple(map(f32, rgb)), f32(power)))

    def add_sphere(self, center, radius, mat_type, rgb, refl, transp=0.0):
        self.objects.append(("sphere", tuple(map(f32, center)), f32(radius),
                             (int(mat_type), tuple(map(f32, rgb)), f32(refl), f32(transp))))
        return len(self.objects) - 1

    def add_triangle(self, v0, v1, v2, mat_type, rgb, refl, transp=0.0):
        self.objects.append(("triangle", tuple(map(f32, v0)), tuple(map(f32, v1)), tuple(map(f32, v2)),
                             (int(mat_type), tuple(map(f32, rgb)), f32(refl), f32(transp))))
        return len(self.objects) - 1

    def add_plane(self, pos, norm, mat_type, rgb, refl, transp=0.0):
        self.objects.append(("plane", tuple(map(f32, pos)), tuple(map(f32, norm)),
                             (int(mat_type), tuple(map(f32, rgb)), f32(refl), f32(transp))))
        return len(self.objects) - 1

    def add_texture(self, tex: Texture) -> int:
        self.textures.append(tex)
        return len(self.textures) - 1

    def set_texture(self, obj, tex, uv):
        self.settex.append((int(obj), int(tex), tuple(map(f32, uv))))

    @property
    def n_spheres(self) -> int:
        return sum(1 for o in self.objects if o[0] == "sphere")

    @property
    def n_triangles(self) -> int:
        return sum(1 for o in self.objects if o[0] == "triangle")

    # ---- serialisation ----
    def write(self, directory: str) -> str:
        """Write ``<name>.scene`` (+ TGA files) into ``directory``; return the scene path."""
        os.makedirs(directory, exist_ok=True)

        def h(x):
            return float(x).hex()

        def texref(t: Optional[Texture]) -> str:
            if t is None or t.argb is None:
                return "-"
            fn = f"{self.name}_{t.name}.tga"
            write_tga(os.path.join(directory, fn), t.argb)
            return fn

        lines = [f"# reflaxman_amd scene '{self.name}'"]
        lines.append("diffuse " + " ".join(h(v) for v in self.diffuse))
        eye, at, fov = self.camera
        lines.append("camera " + " ".join(h(v) for v in (*eye, *at, fov)))
        lines.append("skybox " + texref(self.skybox))
        for (o, r, c, p) in self.lights:
            lines.append("light " + " ".join(h(v) for v in (*o, r, *c, p)))
        # the reference API allows any interleaving; we emit textures first, then objects, then settex
        for t in self.textures:
            lines.append("texture " + texref(t))
        for ob in self.objects:
            mt, rgb, refl, tr = ob[-1]
            if ob[0] == "sphere":
                lines.append("sphere " + " ".join(h(v) for v in (*ob[1], ob[2], mt, *rgb, refl, tr)))
            elif ob[0] == "plane":
                lines.append("plane " + " ".join(h(v) for v in (*ob[1], *ob[2], mt, *rgb, refl, tr)))
            else:
                lines.append("triangle " + " ".join(h(v) for v in (*ob[1], *ob[2], *ob[3], mt, *rgb, refl, tr)))
        for (oi, ti, uv) in self.settex:
            lines.append("settex " + " ".join(h(v) for v in (oi, ti, *uv)))
        path = os.path.join(directory, f"{self.name}.scene")
        with open(path, "w") as f:
            f.write("\n".join(lines) + "\n")
        return path


# ---------------------------------------------------------------------------
# TGA (Texture.cpp:34-137, image_headers.h:4-20)
# ---------------------------------------------------------------------------
def write_tga(path: str, argb: np.ndarray, bpp: int = 32) -> None:
    """Uncompressed type-2 TGA, rows in array order (the reader ignores the origin bit)."""
    h, w = argb.shape
    hdr = struct.pack("<bbbhhbhhhhbb", 0, 0, 2, 0, 0, 0, 0, 0, w, h, bpp, 0)
    a = argb.astype(np.uint32)
    b = (a & 0xFF).astype(np.uint8)
    g = ((a >> 8) & 0xFF).astype(np.uint8)
    r = ((a >> 16) & 0xFF).astype(np.uint8)
    al = ((a >> 24) & 0xFF).astype(np.uint8)
    if bpp == 32:
        px = np.stack([b, g, r, al], axis=-1)
    elif bpp == 24:
        px = np.stack([b, g, r], axis=-1)
    else:
        raise ValueError("bpp must be 24 or 32")
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(px.tobytes())


def read_tga(path: str) -> Optional[np.ndarray]:
    """Texture::loadFromTGAFile semantics (type 2, 24/32 bpp); None on failure."""
    try:
        data = open(path, "rb").read()
    except OSError:
        return None
    if len(data) < 18:
        return None
    idlen, _cmt, itype, _cmorg, cmlen, cmbits, _xo, _yo, w, h, bpp, _desc = struct.unpack("<bbbhhbhhhhbb", data[:18])
    if itype != 2 or bpp not in (24, 32) or w <= 0 or h <= 0:
        return None
    off = 18 + idlen + cmlen * cmbits // 8
    ps = bpp // 8
    n = w * h
    raw = np.frombuffer(data, dtype=np.uint8, count=n * ps, offset=off) if len(data) >= off + n * ps else None
    if raw is None:
        return None
    px = raw.reshape(h, w, ps).astype(np.uint32)
    alpha = px[..., 3] if bpp == 32 else np.full((h, w), 0xFF, np.uint32)
    return (alpha << 24) | (px[..., 2] << 16) | (px[..., 1] << 8) | px[..., 0]


# ---------------------------------------------------------------------------
# deterministic generators
# ---------------------------------------------------------------------------
class Lcg:
    """32-bit Numerical-Recipes LCG used to generate the synthetic scenes."""

    def __init__(self, seed: int):
        self.s = seed & 0xFFFFFFFF

    def next_u32(self) -> int:
        self.s = (1664525 * self.s + 1013904223) & 0xFFFFFFFF
        return self.s

    def uniform(self, lo: float, hi: float) -> float:
        return lo + (hi - lo) * ((self.next_u32() >> 8) / float(1 << 24))


def synth_texture(name: str, w: int, h: int, seed: int) -> Texture:
    """Seeded 32-bpp texture: 16x16-texel colour cells with per-texel noise."""
    rng = Lcg(seed)
    cells_x, cells_y = (w + 15) // 16, (h + 15) // 16
    cell = np.array([[rng.next_u32() for _ in range(cells_x)] for _ in range(cells_y)], dtype=np.uint64)
    ys, xs = np.mgrid[0:h, 0:w]
    base = cell[ys // 16, xs // 16]
    noise_state = (np.arange(w * h, dtype=np.uint64).reshape(h, w) * np.uint64(2654435761) + np.uint64(seed)) & np.uint64(0xFFFFFFFF)
    noise = ((noise_state >> np.uint64(13)) & np.uint64(0x1F)).astype(np.int64)
    out = np.zeros((h, w), dtype=np.uint32)
    for sh in (0, 8, 16):
        ch = ((base >> np.uint64(sh)) & np.uint64(0xFF)).astype(np.int64)
        ch = np.clip(ch // 2 + 64 + noise, 0, 255)
        out |= (ch.astype(np.uint32) << sh)
    alpha = ((noise_state >> np.uint64(3)) & np.uint64(0xFF)).astype(np.uint32)
    return Texture(name, out | (alpha << 24))


DEFAULT_CAMERA = ((7.427, 3.494, -3.773), (6.5981, 3.127, -3.352), 1.05)


def _add_default_spheres(s: SceneDesc) -> None:
    # Render.cpp:39-50
    s.add_sphere((-1.25, 1.5, -0.25), 1.5, METAL, (1.0, 1.0, 1.0), 1.0)
    s.add_sphere((0.15, 1.0, 1.75), 1.0, METAL, (1.0, 1.0, 1.0), 0.95)
    s.add_sphere((-3.0, 0.6, -3.0), 0.6, DIELECTRIC, (1.0, 1.0, 1.0), 0.0)
    s.add_sphere((-0.5, 0.5, -2.5), 0.5, DIELECTRIC, (0.5, 1.0, 0.15), 0.75)
    s.add_sphere((1.0, 0.4, -1.5), 0.4, DIELECTRIC, (0.0, 0.5, 1.0), 1.0)
    s.add_sphere((1.8, 0.4, 0.1), 0.4, METAL, (1.0, 0.65, 0.45), 1.0)
    s.add_sphere((1.7, 0.5, 1.9), 0.5, METAL, (1.0, 0.90, 0.60), 0.75)
    s.add_sphere((0.6, 0.6, 4.2), 0.6, METAL, (0.9, 0.9, 0.9), 0.0)


def _add_ground(s: SceneDesc, tex_index: int) -> None:
    # Render.cpp:52-55: two dielectric triangles forming the 28x20 ground quad
    t1 = s.add_triangle((-14.0, 0.0, -10.0), (-14.0, 0.0, 10.0), (14.0, 0.0, -10.0), DIELECTRIC, (1, 1, 1), 0.95)
    s.set_texture(t1, tex_index, (0.0, 0.0, 0.0, 1.0, 1.0, 0.0))
    t2 = s.add_triangle((-14.0, 0.0, 10.0), (14.0, 0.0, 10.0), (14.0, 0.0, -10.0), DIELECTRIC, (1, 1, 1), 0.95)
    s.set_texture(t2, tex_index, (0.0, 1.0, 1.0, 1.0, 1.0, 0.0))


def _add_sun(s: SceneDesc) -> None:
    s.add_light((11.8e9, 4.26e9, 3.08e9), 3.48e8, (1.0, 1.0, 0.95), 0.85)  # Render.cpp:35


def default_scene(plane_texture: Optional[Texture] = None, skybox: Optional[Texture] = None) -> SceneDesc:
    """Render::loadScene (Render.cpp:25-55); textures absent -> checker."""
    s = SceneDesc("default", (f32(0.95), f32(0.95), f32(1.0), f32(0.15)),
                  (tuple(map(f32, DEFAULT_CAMERA[0])), tuple(map(f32, DEFAULT_CAMERA[1])), f32(DEFAULT_CAMERA[2])))
    s.skybox = skybox
    _add_sun(s)
    _add_default_spheres(s)
    ti = s.add_texture(plane_texture if plane_texture is not None else Texture("himiya", None))
    _add_ground(s, ti)
    return s


def _lcg_spheres(s: SceneDesc, n: int, seed: int = 20261015) -> None:
    """SURVEY.md §8d generator: r~U[0.1,0.6], centre (U[-12,12], r, U[-9,9]), metal/dielectric 50/50,
    colour U[0,1]^3, reflectivity U[0,1]."""
    g = Lcg(seed)
    for _ in range(n):
        r = g.uniform(0.1, 0.6)
        x = g.uniform(-12.0, 12.0)
        z = g.uniform(-9.0, 9.0)
        mt = DIELECTRIC if (g.next_u32() >> 31) else METAL
        rgb = (g.uniform(0, 1), g.uniform(0, 1), g.uniform(0, 1))
        refl = g.uniform(0, 1)
        s.add_sphere((x, r, z), r, mt, rgb, refl)


def synth16_scene(tex_size: int = 512, skybox: bool = False) -> SceneDesc:
    """C3/C4: 8 default + 8 generated spheres, textured ground quad + back wall quad, default sun."""
    s = SceneDesc("synth16" + ("_sky" if skybox else ""), (f32(0.95), f32(0.95), f32(1.0), f32(0.15)),
                  (tuple(map(f32, DEFAULT_CAMERA[0])), tuple(map(f32, DEFAULT_CAMERA[1])), f32(DEFAULT_CAMERA[2])))
    if skybox:
        s.skybox = synth_texture("skybox", 4 * tex_size // 2, 3 * tex_size // 2, 777)
    _add_sun(s)
    _add_default_spheres(s)
    _lcg_spheres(s, 8)
    t_ground = s.add_texture(synth_texture("ground", tex_size, tex_size, 1001))
    t_wall = s.add_texture(synth_texture("wall", tex_size, tex_size, 2002))
    _add_ground(s, t_ground)
    # back wall at x = -14 facing +x (towards the camera), 8 high, z in [-10, 10]
    w1 = s.add_triangle((-14.0, 0.0, -10.0), (-14.0, 8.0, -10.0), (-14.0, 0.0, 10.0), METAL, (0.9, 0.9, 0.9), 0.3)
    s.set_texture(w1, t_wall, (0.0, 0.0, 0.0, 1.0, 1.0, 0.0))
    w2 = s.add_triangle((-14.0, 8.0, -10.0), (-14.0, 8.0, 10.0), (-14.0, 0.0, 10.0), METAL, (0.9, 0.9, 0.9), 0.3)
    s.set_texture(w2, t_wall, (0.0, 1.0, 1.0, 1.0, 1.0, 0.0))
    return s


def stress_scene(n_spheres: int = 4096) -> SceneDesc:
    """C5: n LCG spheres + the ground quad (checker texture), default sun."""
    s = SceneDesc(f"stress{n_spheres}", (f32(0.95), f32(0.95), f32(1.0), f32(0.15)),
                  (tuple(map(f32, DEFAULT_CAMERA[0])), tuple(map(f32, DEFAULT_CAMERA[1])), f32(DEFAULT_CAMERA[2])))
    _add_sun(s)
    _lcg_spheres(s, n_spheres)
    ti = s.add_texture(Texture("himiya", None))
    _add_ground(s, ti)
    return s


def _base(name: str) -> SceneDesc:
    return SceneDesc(name, (f32(0.95), f32(0.95), f32(1.0), f32(0.15)),
                     (tuple(map(f32, DEFAULT_CAMERA[0])), tuple(map(f32, DEFAULT_CAMERA[1])), f32(DEFAULT_CAMERA[2])))


def lights_scene(n_lights: int) -> SceneDesc:
    """Parity scene for the batched light loop: synth16 with n lights -- the sun, then lights at finite
    distance (specular exponents 1 + 3 refl |L| / r far below the sun's) on a ring above the scene, each with
    power 0.8 / n so envColor (the sum of colour x power, Scene.cpp:55) stays near the default's.
    n > 32 takes the kernel's many-lights instantiation (shadow masks in blocks of 32)."""
    s = synth16_scene()
    s.name = f"lights{n_lights}"
    s.lights = []
    _add_sun(s)
    g = Lcg(4040 + n_lights)
    for k in range(n_lights - 1):
        ang = 2.0 * np.pi * k / max(1, n_lights - 1)
        o = (6.0 * np.cos(ang) + g.uniform(-1, 1), g.uniform(4.0, 9.0), 5.0 * np.sin(ang) + g.uniform(-1, 1))
        s.add_light(o, g.uniform(0.2, 1.5), (g.uniform(0.4, 1), g.uniform(0.4, 1), g.uniform(0.4, 1)), 0.8 / n_lights)
    return s


def nolight_scene() -> SceneDesc:
    """The default scene without a light: no shadow rays, ambient and sky only."""
    s = default_scene()
    s.name = "nolight"
    s.lights = []
    return s


def mesh_scene(nx: int = 10, nz: int = 5) -> SceneDesc:
    """More than 64 triangles (2 nx nz): the general (non-small) object loops with two 64-triangle chunks.  A
    height-field ground mesh with per-triangle textures and materials, the 8 default spheres above it."""
    s = _base(f"mesh{2 * nx * nz}")
    _add_sun(s)
    _add_default_spheres(s)
    t0 = s.add_texture(synth_texture("ground", 256, 256, 1001))
    t1 = s.add_texture(Texture("himiya", None))
    g = Lcg(777)
    x0, x1, z0, z1 = -14.0, 14.0, -10.0, 10.0
    hgt = [[0.0 if (i in (0, nx) or j in (0, nz)) else g.uniform(-0.3, 0.3) for j in range(nz + 1)] for i in range(nx + 1)]
    for i in range(nx):
        for j in range(nz):
            xa, xb = x0 + (x1 - x0) * i / nx, x0 + (x1 - x0) * (i + 1) / nx
            za, zb = z0 + (z1 - z0) * j / nz, z0 + (z1 - z0) * (j + 1) / nz
            p00, p01 = (xa, hgt[i][j], za), (xa, hgt[i][j + 1], zb)
            p10, p11 = (xb, hgt[i + 1][j], za), (xb, hgt[i + 1][j + 1], zb)
            mt = DIELECTRIC if (i + j) % 3 else METAL
            rgb = (g.uniform(0.5, 1), g.uniform(0.5, 1), g.uniform(0.5, 1))
            a = s.add_triangle(p00, p01, p10, mt, rgb, g.uniform(0.2, 0.95))
            b = s.add_triangle(p01, p11, p10, mt, rgb, g.uniform(0.2, 0.95))
            tex = t0 if (i + j) % 2 else t1
            u0, u1, v0, v1 = i / nx, (i + 1) / nx, j / nz, (j + 1) / nz
            s.set_texture(a, tex, (u0, v0, u0, v1, u1, v0))
            s.set_texture(b, tex, (u0, v1, u1, v1, u1, v0))
    return s


def planes_scene(n_spheres: int = 0) -> SceneDesc:
    """Planes in a scene (the addPlane extension of Plane.cpp:36-73): the 8 default spheres (or n LCG spheres,
    the general object loops), a textured ground triangle pair, then a dielectric floor plane just below the
    ground (normal not of unit length, as the reference allows) and a metal back-wall plane tilted towards the
    camera.  Objects are added spheres, triangles, planes (the order the kernels visit them)."""
    s = _base(f"planes{n_spheres}" if n_spheres else "planes")
    _add_sun(s)
    if n_spheres:
        _lcg_spheres(s, n_spheres)
    else:
        _add_default_spheres(s)
    ti = s.add_texture(synth_texture("ground", 128, 128, 1001))
    _add_ground(s, ti)
    s.add_plane((0.0, -0.05, 0.0), (0.0, 2.0, 0.0), DIELECTRIC, (0.8, 0.85, 0.9), 0.6)
    s.add_plane((-16.0, 0.0, 0.0), (1.0, 0.05, 0.2), METAL, (0.9, 0.7, 0.5), 0.4)
    return s


SCENES = {
    "default": default_scene,
    "synth16": synth16_scene,
    "synth16_sky": lambda: synth16_scene(skybox=True),
    "stress4096": stress_scene,
    "lights3": lambda: lights_scene(3),
    "lights40": lambda: lights_scene(40),
    "nolight": nolight_scene,
    "mesh100": mesh_scene,
    "planes": planes_scene,
    "planes300": lambda: planes_scene(300),
}


def get_scene(name: str) -> SceneDesc:
    if name.startswith("stress") and name[6:].isdigit():
        return stress_scene(int(name[6:]))
    return SCENES[name]()


def parse_scene_file(path: str) -> SceneDesc:
    """Read a ``.scene`` file written by :meth:`SceneDesc.write` (or by hand)."""
    d = os.path.dirname(os.path.abspath(path))
    s = SceneDesc(os.path.splitext(os.path.basename(path))[0], (0.0, 0.0, 0.0, 0.0), ((0, 0, 0), (0, 0, 1), 1.0))

    def tex(tok: str, name: str) -> Texture:
        if tok == "-":
            return Texture(name, None)
        return Texture(name, read_tga(tok if tok.startswith("/") else os.path.join(d, tok)))

    for line in open(path):
        parts = line.split()
        if not parts or parts[0].startswith("#"):
            continue
        kw, args = parts[0], parts[1:]
        if kw in ("skybox", "texture"):
            t = tex(args[0], args[0])
            if kw == "skybox":
                s.skybox = t
            else:
                s.textures.append(t)
            continue
        v = [float.fromhex(a) if ("0x" in a or "p" in a) else float(a) for a in args]
        if kw == "diffuse":
            s.diffuse = tuple(map(f32, v))
        elif kw == "camera":
            s.camera = (tuple(map(f32, v[0:3])), tuple(map(f32, v[3:6])), f32(v[6]))
        elif kw == "light":
            s.add_light(v[0:3], v[3], v[4:7], v[7])
        elif kw == "sphere":
            s.add_sphere(v[0:3], v[3], int(v[4] != 0), v[5:8], v[8], v[9])
        elif kw == "triangle":
            s.add_triangle(v[0:3], v[3:6], v[6:9], int(v[9] != 0), v[10:13], v[13], v[14])
        elif kw == "plane":
            s.add_plane(v[0:3], v[3:6], int(v[6] != 0), v[7:10], v[10], v[11])
        elif kw == "settex":
            s.set_texture(int(v[0]), int(v[1]), v[2:8])
        else:
            raise ValueError(f"unknown scene keyword {kw!r}")
    return s
