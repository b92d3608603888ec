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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="synth16")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--lib", default="librfx_prof.so")
    ap.add_argument("--regroup", type=int, default=None,
                    help="rfx_renderer_set_regroup setting (large scenes: 0, since only the plain kernel is instrumented)")
    ap.add_argument("--prim", type=int, default=None,
                    help="rfx_renderer_set_prim_masks mode (0: no per-view masks, what a moving camera renders with)")
    a = ap.parse_args()
    path = os.path.join(_build.LIBDIR, "diag", a.lib)
    scene = a.scene
    r = ab.Runner("prof", path, scenes.get_scene(scene), a.width, a.height, a.depth, 1350490027, regroup=a.regroup,
                  prim=a.prim)
    r.render(2)
    assert r.L.rfx_synchronize(r.r) == 0
    buf = (C.c_ulonglong * 16)()
    assert r.L.rfx_debug_prof_read(buf, 1) == 16
    r.render(1)
    assert r.L.rfx_synchronize(r.r) == 0
    assert r.L.rfx_debug_prof_read(buf, 1) == 16
    tot = buf[7]
    cb = (C.c_ulonglong * 32)()
    cull = {}
    if hasattr(r.L, "rfx_debug_cull_read") and r.L.rfx_debug_cull_read(cb, 1) == 32:
        for k, name in ((0, "closest"), (1, "shadow")):
            v = cb[8 * k: 8 * k + 7]
            n = max(v[0], 1)
            cull[name] = {"bundles": v[0], "usable": round(v[1] / n, 3), "live_lanes": round(v[2] / n, 1),
                          "kept_pairs": round(v[3] / n, 2), "valid_pairs": round(v[5] / n, 2),
                          "kept_tris": round(v[4] / n, 2), "valid_tris": round(v[6] / n, 2)}
        v = cb[16:22]
        n = max(v[0], 1)
        cull["closest_large"] = {"bundles": v[0], "usable": round(v[1] / n, 3), "live_lanes": round(v[2] / n, 1),
                                 "kept_chunks": round(v[3] / n, 2), "kept_spheres": round(v[4] / n, 1),
                                 "pair_tests": round(v[5] / n, 1)}
    print(json.dumps({"scene": scene, "lib": os.path.basename(path), "prim_masks": a.prim, "cycles": {k: int(v) for k, v in zip(REGIONS, buf[:8])},
                      "wave_executions": {k: int(v) for k, v in zip(REGIONS, buf[8:])},
                      "share_of_trace": {k: round(v / tot, 4) for k, v in zip(REGIONS, buf[:8])},
                      "cull": cull}))


if __name__ == "__main__":
    main()
