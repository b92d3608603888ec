"""Wave-level utilization of the bounce loop (diagnostic; needs a GPU).

Renders C3 with a RFX_DEBUG_SEGS build (each pixel's color = its trace's segment count) and reports,
for the trace kernel's 8x8-pixel wave tiles, mean segments per lane vs the wave's max -- the fraction
of segment-loop lane slots doing work.
"""
import os
import sys

import numpy as np
import ctypes as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from reflaxman_amd import _build, scenes  # noqa: E402
import ab  # noqa: E402


def main():
    path = os.path.join(_build.LIBDIR, "diag", "librfx_segs.so")
    if not os.path.exists(path):
        path = _build.build_variant("segs", ["RFX_DEBUG_SEGS"])
    W, H = 3840, 2160
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    r = ab.Runner("segs", path, scenes.get_scene(sys.argv[1] if len(sys.argv) > 1 else "synth16"), W, H, depth,
                  1350490027, regroup=0)  # whole traces in one kernel: every pixel's own segment count
    r.render(1)
    assert r.L.rfx_synchronize(r.r) == 0
    rgb = np.empty(W * H * 3, np.float32)
    r.L.rfx_memcpy_d2h(r.r, rgb.ctypes.data_as(C.c_void_p), r.img, rgb.nbytes)
    seg = rgb.reshape(H, W, 3)[:, :, 0]
    t = seg[: H // 8 * 8, : W // 8 * 8].reshape(H // 8, 8, W // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
    mean, mx = t.mean(), t.max(axis=1).mean()
    hist = np.bincount(seg.astype(np.int64).ravel(), minlength=10)
    print({"segments_per_ray": float(mean), "wave_max_mean": float(mx), "loop_lane_util": float(mean / mx),
           "alive_after": {k: int((seg > k).sum()) for k in (1, 2, 3, 4)},
           "hist": hist.tolist(), "wave_max_hist": np.bincount(t.max(axis=1).astype(np.int64), minlength=10).tolist()})


if __name__ == "__main__":
    main()
