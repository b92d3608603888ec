"""The RNG pre-pass's integer accept test (rfx_kernels.hip triple / sphere_n) decides exactly as the reference's float
test (src/common/Vector3.cpp:182-185) outside its shell, over all 2^45 triples of 15-bit draws.

tests/native/sphere_shell.c walks every (k1, k2) and both sides of k3 (8 threads, about 20 s here) and reports the
largest N = sum (2k - 32767)^2 of a float-accepted triple and the smallest N of a rejected one; the device constant
kSphereShell must cover both distances from 32767^2.
"""
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R2 = 32767 * 32767


def _device_shell():
    src = open(os.path.join(ROOT, "reflaxman_amd", "csrc", "rfx_kernels.hip")).read()
    return int(re.search(r"constexpr uint32_t kSphereShell = (\d+)u;", src).group(1))


@pytest.fixture(scope="module")
def shell_run(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("shell") / "sphere_shell")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fopenmp",
                    os.path.join(ROOT, "tests", "native", "sphere_shell.c"), "-o", exe], check=True)
    r = subprocess.run([exe, "1"], capture_output=True, text=True, env=dict(os.environ, OMP_NUM_THREADS="8"))
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout)


def test_every_triple_off_the_shell_decides_like_the_float_test(shell_run):
    res = shell_run
    assert res["pairs"] == 1 << 30 and res["r2"] == R2
    shell = _device_shell()
    assert res["accepted_max_n"] - R2 <= shell and R2 - res["rejected_min_n"] <= shell, res
    # the measured extremes (a change of the float evaluation would move them)
    assert (res["accepted_max_n"] - R2, R2 - res["rejected_min_n"]) == (298, 174)
    # about pi / 6 of the cube accepted
    assert abs(res["accepted"] / 2.0 ** 45 - np.pi / 6) < 1e-4


def test_sphere_n_mod_2_32_is_the_centred_sum():
    """sphere_n evaluates 4 sum k^2 - 131068 sum k + 3 * 32767^2 in uint32: the same number as sum (2k - 32767)^2."""
    rng = np.random.default_rng(5)
    k = rng.integers(0, 1 << 15, size=(1_000_000, 3), dtype=np.uint64)
    k = np.concatenate([k, np.array([[0, 0, 0], [32767, 32767, 32767], [0, 32767, 16383], [16384, 16383, 16384]],
                                    np.uint64)])
    with np.errstate(over="ignore"):
        q = (k * k).sum(1).astype(np.uint32)
        t = k.sum(1).astype(np.uint32)
        n = np.uint32(4) * q - np.uint32(131068) * t + np.uint32(3 * R2)
    exact = ((2 * k.astype(np.int64) - 32767) ** 2).sum(1)
    assert exact.max() < 1 << 32
    assert np.array_equal(n.astype(np.int64), exact)


def test_integer_and_float_tests_agree_on_samples():
    """A direct sample of the claim, independent of the C walk: random triples and triples near the sphere."""
    rng = np.random.default_rng(11)
    half = np.float32(np.float32(0x7FFF) / np.float32(2))
    x_of = (np.arange(1 << 15, dtype=np.float32) / half - np.float32(1)).astype(np.float32)
    k = rng.integers(0, 1 << 15, size=(2_000_000, 3))
    # plus triples with k3 chosen so that N is within a few thousand of 32767^2
    k12 = rng.integers(0, 1 << 15, size=(200_000, 2))
    v12 = ((2 * k12 - 32767) ** 2).sum(1)
    room = R2 - v12
    ok = room > 0
    v3 = np.floor(np.sqrt(room[ok])).astype(np.int64)
    v3 = v3 - (v3 % 2 == 0)  # odd: v = 2k - 32767
    k3 = (v3 + 32767) // 2 + rng.integers(-2, 3, size=v3.shape)
    k3 = np.clip(k3, 0, 32767)
    k = np.concatenate([k, np.column_stack([k12[ok], k3])])
    x = x_of[k]
    with np.errstate(over="ignore"):
        s = (x[:, 0] * x[:, 0] + x[:, 1] * x[:, 1]).astype(np.float32)
        s = (s + (x[:, 2] * x[:, 2]).astype(np.float32)).astype(np.float32)
    float_acc = ~(s > np.float32(1))
    n = ((2 * k - 32767) ** 2).sum(1)
    shell = _device_shell()
    off = np.abs(n - R2) > shell
    assert off.sum() > 2_000_000
    assert np.array_equal(float_acc[off], n[off] < R2)


def test_pre_pass_code_has_no_byte_dot_products(tmp_path):
    """Guard against the ROCm 7.2 fold sphere_n's comment describes: the RNG kernels' device code (hipcc -S of
    rfx_kernels.hip with the library's flags) holds no v_dot4_u32_u8, which would square one byte of each draw only."""
    import shutil
    from reflaxman_amd import _build
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    out = tmp_path / "k.s"
    subprocess.run([hipcc, *_build.FLAGS, "--cuda-device-only", "-S",
                    os.path.join(ROOT, "reflaxman_amd", "csrc", "rfx_kernels.hip"), "-o", str(out)],
                   check=True, capture_output=True)
    asm = out.read_text()
    assert "v_mad_u32_u24" in asm
    assert "v_dot4_u32_u8" not in asm


def _jump(n):
    a, c, A, C = 214013, 2531011, 1, 0
    while n:
        if n & 1:
            A, C = (a * A) & 0xFFFFFFFF, (a * C + c) & 0xFFFFFFFF
        c, a, n = (a * c + c) & 0xFFFFFFFF, (a * a) & 0xFFFFFFFF, n >> 1
    return np.uint32(A), np.uint32(C)


def test_full_frame_streams_reach_the_shell():
    """The float fallback is not dead code for the parity tests: the stream a renderer starts from its default seed
    (1350490027, the C3 / C4 full-frame cases' frame 0) puts triples on the shell within the C3 frame's ~15.8 M
    triples, so those frames' hashes check it.  Thread starts by doubling (jumps of 48 draws), then 16 triples each."""
    seed, nthreads = 1350490027, 4054 * 256  # C3: 4,054 pre-pass blocks of 256 threads
    S = np.empty(nthreads, np.uint32)
    S[0] = seed
    k = 1
    with np.errstate(over="ignore"):
        while k < nthreads:
            A, C = _jump(48 * k)
            m = min(k, nthreads - k)
            S[k:k + m] = A * S[:m] + C
            k *= 2
        s, shell = S.copy(), 0
        for _ in range(16):
            n = np.zeros(nthreads, np.int64)
            for _ in range(3):
                s = np.uint32(214013) * s + np.uint32(2531011)
                n += (2 * ((s >> 16) & 0x7FFF).astype(np.int64) - 32767) ** 2
            shell += int((np.abs(n - R2) <= _device_shell()).sum())
    assert shell >= 10, shell  # 19 for kSphereShell = 1024
