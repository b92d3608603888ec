"""bench.py helpers that need no GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_strong_scaling_baseline_is_the_committed_one_gpu_c4_line():
    b = bench.one_gpu_line("c4", 7680, 4320, 8)
    assert b is not None and b["unit"] == "Mrays/s" and b["value"] > 0
    assert b["source"].startswith(os.path.join("profiles", "r02", "configs"))
    assert bench.one_gpu_line("c4", 640, 360, 8) is None  # another frame: no baseline


def test_cpu_sample_strides_cover_every_config():
    assert set(bench.CPU_STRIDE) == set(bench.CONFIGS)


def test_weak_and_strong_frame_sizes():
    assert bench.frame_size(1, 3840, 2160, "weak") == (3840, 2160)
    assert bench.frame_size(8, 7680, 4320, "strong") == (7680, 4320)
    w, h = bench.frame_size(4, 3840, 2160, "weak")
    assert (w, h) == (7680, 4320)
