"""Where the trace kernel's wave time goes (diagnostic; needs a GPU).

Renders C3 with a RFX_DEBUG_PROF build, which sums s_memtime deltas per region of the bounce segment
(sphere loop, triangle loop, winner re-derivation, light loop, its shadow any-hit, material, sky) and
of the whole trace, and prints each region's share of the trace total.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from reflaxman_amd import _build, scenes  # noqa: E402
import ab  # noqa: E402

REGIONS = ["sphere_loop", "triangle_loop", "winner", "light_loop", "shadow_anyhit", "material", "sky", "trace"]


def main():
    path = os.path.join(_build.LIBDIR, "diag", sys.argv[2] if len(sys.argv) > 2 else "librfx_prof.so")
    scene = sys.argv[1] if len(sys.argv) > 1 else "synth16"
    r = ab.Runner("prof", path, scenes.get_scene(scene), 3840, 2160, 8, 1350490027)
    r.render(2)
    assert r.L.rfx_synchronize(r.r) == 0
    buf = (C.c_ulonglong * 16)()
    assert r.L.rfx_debug_prof_read(buf, 1) == 16
    r.render(1)
    assert r.L.rfx_synchronize(r.r) == 0
    assert r.L.rfx_debug_prof_read(buf, 1) == 16
    tot = buf[7]
    cb = (C.c_ulonglong * 16)()
    cull = {}
    if hasattr(r.L, "rfx_debug_cull_read") and r.L.rfx_debug_cull_read(cb, 1) == 16:
        for k, name in ((0, "closest"), (1, "shadow")):
            v = cb[8 * k: 8 * k + 7]
            n = max(v[0], 1)
            cull[name] = {"bundles": v[0], "usable": round(v[1] / n, 3), "live_lanes": round(v[2] / n, 1),
                          "kept_pairs": round(v[3] / n, 2), "valid_pairs": round(v[5] / n, 2),
                          "kept_tris": round(v[4] / n, 2), "valid_tris": round(v[6] / n, 2)}
    print(json.dumps({"scene": scene, "lib": os.path.basename(path), "cycles": {k: int(v) for k, v in zip(REGIONS, buf[:8])},
                      "wave_executions": {k: int(v) for k, v in zip(REGIONS, buf[8:])},
                      "share_of_trace": {k: round(v / tot, 4) for k, v in zip(REGIONS, buf[:8])},
                      "cull": cull}))


if __name__ == "__main__":
    main()
