"""Build librfx.so (HIP kernels + C-ABI) in-tree for gfx950.

The library is compiled with the flags the parity contract needs:
``-ffp-contract=off`` (no FMA contraction, host and device), no fast-math,
IEEE-correct fp32 division/sqrt on the device and f32 denormals preserved.
"""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "librfx.so")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")

SOURCES = ["rfx_kernels.hip", "rfx_host.cpp"]
HEADERS = ["rfx_math.h", "rfx_powf.h", "rfx_types.h"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

FLAGS = [
    "-O3", "-std=c++17", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
    "-fno-slp-vectorize",  # auto-packing v3 code costs more v_mov than it saves (tools/ab.py: -7% trace time)
    "-fPIC", "-shared", "-Wall", "-Wno-unknown-pragmas",
]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build librfx.so")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "rfx.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build_variant(name: str, defines, verbose: bool = False) -> str:
    """Compile a variant librfx_<name>.so with extra -D defines / compiler flags (A/B timing builds, tools/ab.py)."""
    out = os.path.join(LIBDIR, "variants", f"librfx_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    extra = [d if d.startswith("-") else f"-D{d}" for d in defines]  # "-..." entries are compiler flags
    cmd = [hipcc(), *FLAGS, *extra, *[os.path.join(CSRC, s) for s in SOURCES], "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"variant {name} build failed:\n" + r.stdout + r.stderr)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile librfx.so if missing or older than its sources; return its path."""
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = LIB + ".tmp"
    cmd = [hipcc(), *FLAGS, *[os.path.join(CSRC, s) for s in SOURCES], "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("librfx.so build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    if verbose:
        print(r.stderr)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
