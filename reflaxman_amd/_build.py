"""Build librfx.so (HIP kernels + C-ABI) in-tree for gfx950.

The library is compiled with the flags the parity contract needs:
``-ffp-contract=off`` (no FMA contraction, host and device), no fast-math,
IEEE-correct fp32 division/sqrt on the device and f32 denormals preserved.
"""
from __future__ import annotations

import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "librfx.so")
ROOT = os.path.dirname(HERE)
INCLUDE = os.path.join(ROOT, "include")

# the trace kernel families compile as separate TUs in parallel (one hipcc per source), then link
SOURCES = ["rfx_kernels.hip", "rfx_host.cpp", "rfx_group.cpp", "rfx_trace_plain_park.hip"] + [
    f"rfx_trace_{m}_{s}.hip" for m in ("plain", "ssaa", "lanes", "chunks", "block") for s in ("fast", "stats")]
HEADERS = ["rfx_math.h", "rfx_powf.h", "rfx_types.h", "rfx_trace.h", "rfx_internal.h"]
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"

FLAGS = [
    "-O3", "-std=c++17", f"--offload-arch={ARCH}",
    "-ffp-contract=off", "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt", "-fno-gpu-flush-denormals-to-zero",
    "-fno-slp-vectorize",  # auto-packing v3 code costs more v_mov than it saves (tools/ab.py: -7% trace time)
    "-fPIC", "-Wall", "-Wno-unknown-pragmas",
]
JOBS = min(8, os.cpu_count() or 1)


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build librfx.so")


def _sources_digest() -> str:
    """SHA-256 over the compiler flags and the contents of every source and header the library is built from."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for d in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(INCLUDE, "rfx.h")]:
        h.update(os.path.basename(d).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


DIGEST = LIB + ".src.sha256"  # the digest of the sources the in-tree librfx.so was built from


def _stale() -> bool:
    """Content-based: the library is stale when it is missing or was built from other sources (file times are not
    compared -- a copied tree, e.g. on a GPU box, keeps the library it came with)."""
    if not os.path.exists(LIB) or not os.path.exists(DIGEST):
        return True
    with open(DIGEST) as f:
        return f.read().strip() != _sources_digest()


def _compile_link(out: str, extra, objdir: str) -> str:
    """hipcc -c every source into objdir (in parallel), then hipcc -shared into out; returns compiler stderr."""
    os.makedirs(objdir, exist_ok=True)

    def one(src):
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        # compiled from inside csrc/ by relative name, with the tree's root mapped to '.' and a fixed compilation-unit
        # id (HIP derives the default from the input path): the code objects carry nothing of the build directory, so
        # the device code -- and its hash, _lib.device_sha256, which keys profiles/pmc -- is the same wherever the tree
        # is built
        cmd = [hipcc(), *FLAGS, *extra, f"-ffile-prefix-map={ROOT}=.", f"-cuid=rfx_{os.path.splitext(src)[0]}", "-c", src,
               "-o", os.path.abspath(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=CSRC)
        if r.returncode != 0:
            raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        return obj, r.stderr

    with ThreadPoolExecutor(JOBS) as ex:
        res = list(ex.map(one, SOURCES))
    cmd = [hipcc(), *FLAGS, "-shared", *[o for o, _ in res], "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    return "".join(e for _, e in res)


def build_variant(name: str, defines, verbose: bool = False) -> str:
    """Compile a variant librfx_<name>.so with extra -D defines / compiler flags (A/B timing builds, tools/ab.py)."""
    out = os.path.join(LIBDIR, "variants", f"librfx_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    extra = [d if d.startswith("-") else f"-D{d}" for d in defines]  # "-..." entries are compiler flags
    try:
        _compile_link(out, extra, os.path.join(LIBDIR, "variants", "obj_" + name))
    except RuntimeError as e:
        raise RuntimeError(f"variant {name}: {e}") from None
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile librfx.so if missing or built from other sources; return its path."""
    if not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    # the digest of the sources as they are when compilation starts: a file edited during the build leaves the
    # library recorded under the older digest, so the next build() sees it stale
    digest = _sources_digest()
    tmp = LIB + ".tmp"
    err = _compile_link(tmp, [], os.path.join(LIBDIR, "obj"))
    if verbose:
        print(err)
    os.replace(tmp, LIB)
    with open(DIGEST, "w") as f:
        f.write(digest + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))
