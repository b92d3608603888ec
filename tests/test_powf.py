"""The device powf restatement (reflaxman_amd/csrc/rfx_powf.h) is bit-identical to this host's
glibc powf -- the function the reference calls at Scene.cpp:175 and :196."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("powf") / "powf_check")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wno-unknown-pragmas",
                    "-pthread", "-I" + os.path.join(ROOT, "reflaxman_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "powf_check.cpp"), "-o", exe, "-lm"], check=True)
    return exe


def test_powf_bitexact_vs_libm(checker):
    # Fresnel site: every 7th float in [0, 1] with y = 3; specular site: 2e7 random (x, y); specials
    r = subprocess.run([checker, "20000000", "7"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


def test_powf_restatement_matches_reference_kat(checker, tmp_path):
    """kat_pow.npz: powf at both call sites' domains as the reference computed it (tools/gen_golden.py,
    refharness kat_pow).  The fixture equals this host's live glibc powf and the product restatement."""
    import ctypes
    import numpy as np
    g = np.load(os.path.join(ROOT, "tests", "golden", "kat_pow.npz"))
    inp = np.ascontiguousarray(g["inp"], np.float32)
    libm = ctypes.CDLL("libm.so.6")
    libm.powf.restype = ctypes.c_float
    libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    live = np.array([libm.powf(float(x), float(y)) for x, y in inp], np.float32)
    assert live.tobytes() == g["out"].tobytes()
    fi, fo = tmp_path / "in.bin", tmp_path / "out.bin"
    inp.tofile(fi)
    subprocess.run([checker, "-f", str(fi), str(fo)], check=True)
    ours = np.fromfile(fo, np.float32)
    assert ours.tobytes() == g["out"].tobytes(), np.argwhere(ours != g["out"])[:5]


def test_fresnel_cube_form_every_float(checker):
    """Scene.cpp:196's powf(x, 3) as the bounce loop evaluates it -- the double cube where every value within 2^-32 of
    it rounds alike, glibc's algorithm elsewhere (rfx_powf.h powf_cube_fast) -- equals the live libm on every float
    in [0, 1] (the term's whole domain: x = 1 - cosA with cosA clamped to [0, 1])."""
    r = subprocess.run([checker, "-cube"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout
