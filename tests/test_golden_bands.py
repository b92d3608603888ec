"""The banded golden generator (tools/gen_golden.py banded_frame, oracle/_ref/refharness bandss) against the reference's
own Render::renderBegin + renderNext (refharness render) on small frames: one-sample, SSAA and a later frame of the
stream, split into bands of a few rows.  The full-size hashes of C5, C2 depth 1 and the screenshot workload are made
this way.  Needs the reference build (this container); skipped where oracle/_ref/refharness is absent."""
import os
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "refharness")
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.skipif(not os.path.exists(HARNESS), reason="needs oracle/_ref/refharness (the reference build)")


@pytest.mark.parametrize("scene,W,H,depth,ss,frames", [
    ("default", 24, 17, 6, 1, 1),
    ("default", 20, 13, 8, 2, 2),
    ("default", 9, 7, 20, 4, 1),
    ("planes", 16, 11, 6, 3, 2),
])
def test_bands_equal_render_next(scene, W, H, depth, ss, frames):
    import gen_golden
    from reflaxman_amd import scenes
    with tempfile.TemporaryDirectory() as tmp:
        arg = "default" if scene == "default" else scenes.get_scene(scene).write(os.path.join(tmp, "sc"))
        rgb, argb = gen_golden.render_case(tmp, arg, W, H, depth, ss, False, frames, gen_golden.DEFAULT_SEED, 0)
        brgb, bargb = gen_golden.banded_frame(tmp, arg, W, H, depth, ss, frames - 1, gen_golden.DEFAULT_SEED,
                                              workers=4, band_rows=3)
    assert brgb.tobytes() == rgb.tobytes()
    assert np.array_equal(bargb, argb)
