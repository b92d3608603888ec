"""The drop-in boundary against the reference's only real caller, src/common/Pulse.cpp (unmodified).

include/reflaxman/dropin/{Render,Scene}.h replace the reference's Render.h / Scene.h; the caller keeps its
own value types, asset IO and camera motion (Camera::proceedControl / inMotion, Pulse.cpp:96,108) and links
librfx.so instead of the renderer's .cpp files (tools/pulse_build.py).  A headless platform
(tests/native/pulse_headless.cpp) drives Pulse's screenshot flow: F2, 800x600, SSAA 2x2, depth 20.

* CPU (build container, needs /root/reference): Pulse.cpp and the caller's sources compile and link against
  the drop-in headers -- the compile-only proof a maintainer needs.
* GPU: the drop-in Pulse binary (built in-tree by __graft_entry__.build()) writes a screenshot whose BMP file
  equals, byte for byte, the one the reference's own Pulse + CPU renderer wrote (tests/golden/manifest.json
  pulse_screenshot_800x600_ss2, tools/gen_golden.py).
"""
import hashlib
import os
import subprocess
import sys

import pytest

from helpers import manifest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "tests", "native", "_build", "pulse_dropin")


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/common"), reason="needs the reference sources")
def test_pulse_compiles_against_dropin_headers(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pulse_build
    exe = pulse_build.build("dropin", str(tmp_path / "pulse_dropin"))
    assert os.path.getsize(exe) > 0


@pytest.mark.skipif(not os.path.isdir("/root/reference/src/common"), reason="needs the reference sources")
def test_dropin_scene_revisions_and_moved_handles(tmp_path):
    """dropin/Scene.h: every Scene state has its own revision (a re-assigned Scene never repeats an earlier one, so
    Render::renderNext re-uploads it), and a moved Scene's Triangle handles act on the Scene they now belong to.  Host
    calls only: runs on the CPU (tests/native/dropin_scene_revision.cpp)."""
    ref = "/root/reference/src/common"
    src = tmp_path / "src"
    src.mkdir()
    keep = ["Color", "Material", "OmniLight", "Texture", "Vector3", "trace_math", "Matrix33"]
    for n in [f + e for f in keep for e in (".h", ".cpp")] + ["image_headers.h", "defaults.h"]:
        if os.path.exists(os.path.join(ref, n)):
            os.symlink(os.path.join(ref, n), src / n)
    lib = os.path.join(ROOT, "reflaxman_amd", "lib")
    exe = str(tmp_path / "rev")
    cmd = ["g++", "-std=c++11", "-O2", "-ffp-contract=off", "-DNDEBUG", "-w", "-I", str(src),
           "-I", os.path.join(ROOT, "include", "reflaxman", "dropin"), "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "native", "dropin_scene_revision.cpp"),
           *[str(src / (f + ".cpp")) for f in keep], "-L", lib, "-lrfx", f"-Wl,-rpath,{lib}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


@pytest.mark.gpu
def test_pulse_screenshot_matches_reference(tmp_path):
    c = manifest()["cases"]["pulse_screenshot_800x600_ss2"]
    if not os.path.exists(DROPIN):
        pytest.fail("tests/native/_build/pulse_dropin missing: run __graft_entry__.build() where /root/reference exists")
    env = {**os.environ, "RFX_SPHERE_SEED": str(c["RFX_SPHERE_SEED"]), "RFX_JITTER_SEED": str(c["RFX_JITTER_SEED"])}
    out = str(tmp_path) + "/"
    r = subprocess.run([DROPIN, out, str(c["res_key"]), str(c["ss_key"])], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    path = r.stdout.strip()
    assert os.path.basename(path) == c["file"]
    data = open(path, "rb").read()
    assert len(data) == c["bytes"]
    assert hashlib.sha256(data).hexdigest() == c["sha_bmp"]


@pytest.mark.gpu
def test_pulse_screenshot_on_a_device_group(tmp_path):
    """The same screenshot with the drop-in's frames cut into row bands over a group of 3 members (RFX_DEVICES; all
    device 0 on the one-GPU box): byte-identical BMP."""
    c = manifest()["cases"]["pulse_screenshot_800x600_ss2"]
    if not os.path.exists(DROPIN):
        pytest.fail("tests/native/_build/pulse_dropin missing: run __graft_entry__.build() where /root/reference exists")
    env = {**os.environ, "RFX_SPHERE_SEED": str(c["RFX_SPHERE_SEED"]), "RFX_JITTER_SEED": str(c["RFX_JITTER_SEED"]),
           "RFX_DEVICES": "0,0,0"}
    r = subprocess.run([DROPIN, str(tmp_path) + "/", str(c["res_key"]), str(c["ss_key"])], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    data = open(r.stdout.strip(), "rb").read()
    assert hashlib.sha256(data).hexdigest() == c["sha_bmp"]


@pytest.mark.gpu
@pytest.mark.parametrize("case,devices,policy", [("pulse_screenshot_800x600_ss128", None, "frame"),
                                                  ("pulse_screenshot_800x600_ss128", None, "span"),
                                                  ("pulse_screenshot_800x600_ss128", "0,0,0", "frame"),
                                                  ("pulse_screenshot_1920x1080_ss128", None, "frame"),
                                                  ("pulse_screenshot_1920x1080_ss128", "0,0,0", "frame")])
def test_pulse_screenshot_128x128_samples(tmp_path, case, devices, policy):
    """Pulse's screenshot with 128x128 SSAA (menu key 8; Pulse.cpp:10-34) at 800x600 (7.9e9 samples) and at 1920x1080,
    the reference's ReadMe image (ReadMe.md:30-32; 3.4e10 samples): more than 2^32, which the renderer splits into
    launches (rfx_render_frame) or row-span passes (a device group).  The BMP equals, byte for byte, the reference's frame
    written by the reference's Texture::saveToFile (tools/gen_golden.py; the route is pinned to the reference Pulse's own
    BMP at 2x2)."""
    c = manifest()["cases"][case]
    if not os.path.exists(DROPIN):
        pytest.fail("tests/native/_build/pulse_dropin missing: run __graft_entry__.build() where /root/reference exists")
    env = {k: v for k, v in os.environ.items() if k != "RFX_DEVICES"}
    env.update({"RFX_SPHERE_SEED": str(c["RFX_SPHERE_SEED"]), "RFX_JITTER_SEED": str(c["RFX_JITTER_SEED"]),
                "RFX_DROPIN_POLICY": policy, **({"RFX_DEVICES": devices} if devices else {})})
    r = subprocess.run([DROPIN, str(tmp_path) + "/", str(c["res_key"]), str(c["ss_key"])], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    data = open(r.stdout.strip(), "rb").read()
    assert len(data) == c["bytes"]
    assert hashlib.sha256(data).hexdigest() == c["sha_bmp"]


def run_frames(tmp_path, c, devices=None, policy="frame"):
    """A non-Pulse caller of the drop-in Render: each frame of case c in one renderNext(W*H) call."""
    if not os.path.exists(DROPIN):
        pytest.fail("tests/native/_build/pulse_dropin missing: run __graft_entry__.build() where /root/reference exists")
    env = {k: v for k, v in os.environ.items() if k != "RFX_DEVICES"}
    env.update({"RFX_SPHERE_SEED": str(c["sphere_seed"]), "RFX_JITTER_SEED": str(c.get("jitter_seed", 0)),
                "RFX_DROPIN_POLICY": policy, **({"RFX_DEVICES": devices} if devices else {})})
    out = str(tmp_path / "frame")
    r = subprocess.run([DROPIN, out, "frames", str(c["W"]), str(c["H"]), str(c["depth"]), str(c["ss"]),
                        str(int(c["additive"])), str(c["frames"])], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
    f32 = open(out + ".f32", "rb").read()
    argb = open(out + ".argb", "rb").read()
    return hashlib.sha256(f32).hexdigest(), hashlib.sha256(argb).hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("devices,policy", [(None, "frame"), ("0,0", "frame"), ("0,0,0", "span")])
def test_single_call_screenshot_frame(tmp_path, devices, policy):
    """The reference's screenshot workload (Full HD, 4x4 SSAA, depth 20: Pulse.cpp:156-178, defaults.h:9) rendered by
    a caller that covers the frame with one renderNext(W*H) -- on one device, and cut into row bands over a device
    group (RFX_DEVICES; all members on device 0 on the one-GPU box) under either policy: SHA-256 of imagePixel's floats
    and of copyImage's ARGB8 equal the reference's full frame (tools/gen_golden.py, banded refharness)."""
    c = manifest()["cases"]["hash_default_1920x1080_d20_ss4"]
    assert run_frames(tmp_path, c, devices, policy) == (c["sha_f32"], c["sha_argb"])


@pytest.mark.gpu
def test_single_call_additive_frames_on_a_device_group(tmp_path):
    """Two additive SSAA-2 frames, each in one renderNext(W*H) call, over a 2-member group: the second frame
    accumulates onto the first across the members' bands; equal to the reference's stored golden."""
    import numpy as np
    from helpers import GOLDEN
    key = "render_default_96x64_d4_ss2_add2"
    c = manifest()["cases"][key]
    g = np.load(os.path.join(GOLDEN, key + ".npz"))
    # imagePixel divides by additiveCounter, as the reference (Render.cpp:103-114); the golden was read the same way
    assert run_frames(tmp_path, c, "0,0") == (hashlib.sha256(g["rgb"].tobytes()).hexdigest(),
                                               hashlib.sha256(g["argb"].tobytes()).hexdigest())


def run_session(tmp_path, c, policy, hash_frames=True, devices=None):
    """The interactive session of tests/native/pulse_headless.cpp through the drop-in; returns the parsed frame lines."""
    if not os.path.exists(DROPIN):
        pytest.fail("tests/native/_build/pulse_dropin missing: run __graft_entry__.build() where /root/reference exists")
    env = {**os.environ, "RFX_SPHERE_SEED": str(c["RFX_SPHERE_SEED"]), "RFX_JITTER_SEED": str(c["RFX_JITTER_SEED"]),
           "RFX_DROPIN_POLICY": policy, **({"RFX_DEVICES": devices} if devices else {})}
    cmd = [DROPIN, str(tmp_path) + "/", "session", str(c["W"]), str(c["H"]), str(c["tick_us"])]
    r = subprocess.run(cmd + ([] if hash_frames else ["nohash"]), capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return [l.split() for l in r.stdout.splitlines() if l.startswith("frame ")]


@pytest.mark.gpu
@pytest.mark.parametrize("tick", [1000, 2000])
@pytest.mark.parametrize("policy", ["frame", "span"])
def test_pulse_interactive_session_matches_reference(tmp_path, tick, policy):
    """Pulse's interactive loop (Pulse.cpp:102-154) through the drop-in, against the same session through the
    reference's CPU renderer: still additive frames at depth 15, a key press that abandons a frame after 7 chunks,
    motion frames in block preview at depth 4 (sampleNum held at -1, or walked down to -8 by the slower fake clock),
    release, deceleration, still frames again.  Every completed frame, read back as the window reads it
    (getRenderImagePixel over the client area), hashes to the reference's; the per-frame chunk counts are the same.
    Policy "frame" renders each frame whole at its first renderNext (and settles the abandoned one exactly); "span"
    renders each chunk as it comes."""
    c = manifest()["cases"][f"pulse_session_640x480_tick{tick}"]
    frames = run_session(tmp_path, c, policy)
    assert [f[7] for f in frames] == c["hashes"]
    assert [int(f[3]) for f in frames] == c["execs"]


@pytest.mark.gpu
def test_pulse_interactive_session_on_a_device_group(tmp_path):
    """The interactive session with RFX_DEVICES=0,0 (a 2-member group on the one-GPU box): the still frames
    (sampleNum 1, additive: accumulation over the group's bands) go through rfx_group_render_frame, the motion frames
    (block preview) and the settled abandoned frame through member 0; every frame hashes to the reference's."""
    c = manifest()["cases"]["pulse_session_640x480_tick2000"]
    frames = run_session(tmp_path, c, "frame", devices="0,0")
    assert [f[7] for f in frames] == c["hashes"]
