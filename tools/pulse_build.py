#!/usr/bin/env python3
"""Build the reference's own application controller (src/common/Pulse.cpp, unmodified) headless, two ways.

    python tools/pulse_build.py reference OUT   # Pulse + the reference's CPU renderer (Render.cpp, Scene.cpp, ...)
    python tools/pulse_build.py dropin OUT      # Pulse + include/reflaxman/dropin/{Render,Scene}.h + librfx.so

Needs /root/reference (this container).  Nothing of the reference is copied: the drop-in build compiles the
caller-side sources where they lie, through a scratch directory of symbolic links from which the reference's
Render.h / Scene.h and the renderer's .cpp files are absent -- which is the change a maintainer makes when
switching the build over.  The drop-in binary links librfx.so through a relative rpath,
so a binary built here runs from the same tree on the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/src/common"
FLAGS = ["-std=c++11", "-O2", "-ffp-contract=off", "-fno-fast-math", "-DNDEBUG", "-w"]
# the caller's own sources that stay in the build (value types, asset IO, camera motion, the app controller)
CALLER = ["Pulse", "BasePlatformInterface", "Camera", "Color", "Material", "Matrix33", "OmniLight", "Texture",
          "Vector3", "trace_math"]
HEADERS_ONLY = ["defaults.h", "image_headers.h"]
RENDERER = ["Render", "Scene", "SceneObject", "Skybox", "Sphere", "Triangle", "Plane"]


def build(kind: str, out: str) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    main = os.path.join(ROOT, "tests", "native", "pulse_headless.cpp")
    with tempfile.TemporaryDirectory() as tmp:
        if kind == "reference":
            # the seed hook makes the reference's per-TU rand() seeds explicit (RFX_SPHERE_SEED / RFX_JITTER_SEED)
            seed = os.path.join(tmp, "ref_seed.o")
            subprocess.run(["gcc", "-O2", "-c", os.path.join(ROOT, "oracle", "ref_seed.c"), "-o", seed], check=True)
            srcs = [os.path.join(REF, f + ".cpp") for f in CALLER + RENDERER]
            cmd = ["g++", *FLAGS, "-include", os.path.join(ROOT, "oracle", "ref_seed_shim.h"), "-I", REF, main, *srcs,
                   seed, "-o", out, "-lm"]
        elif kind == "dropin":
            src = os.path.join(tmp, "src")
            os.makedirs(src)
            names = [f + ext for f in CALLER for ext in (".h", ".cpp") if os.path.exists(os.path.join(REF, f + ext))]
            for n in names + HEADERS_ONLY:
                os.symlink(os.path.join(REF, n), os.path.join(src, n))
            srcs = [os.path.join(src, f + ".cpp") for f in CALLER]
            lib = os.path.join(ROOT, "reflaxman_amd", "lib")
            rpath = os.path.relpath(lib, os.path.dirname(os.path.abspath(out)))
            cmd = ["g++", *FLAGS, "-I", src, "-I", os.path.join(ROOT, "include", "reflaxman", "dropin"),
                   "-I", os.path.join(ROOT, "include"), main, *srcs, "-o", out,
                   "-L", lib, "-lrfx", f"-Wl,-rpath,$ORIGIN/{rpath}"]
        else:
            raise ValueError(kind)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(" ".join(cmd) + "\n" + r.stdout + r.stderr)
    return out


if __name__ == "__main__":
    print(build(sys.argv[1], sys.argv[2]))
