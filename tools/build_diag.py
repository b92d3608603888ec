"""Build the diagnostic librfx variants tools/regionprof.py and tools/segstats.py load (CPU; hipcc only).

    python tools/build_diag.py      # -> reflaxman_amd/lib/diag/librfx_{prof,segs,waves}.so

librfx_prof.so: RFX_DEBUG_PROF (s_memtime region sums and bundle cull statistics);
librfx_segs.so: RFX_DEBUG_SEGS (each trace's segment count replaces its colour);
librfx_waves.so: RFX_DEBUG_WAVES (each plain-mode wave's start and end time, tools/wave_timeline.py).
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from reflaxman_amd import _build  # noqa: E402

DIAG = {"prof": ["RFX_DEBUG_PROF"], "segs": ["RFX_DEBUG_SEGS"], "waves": ["RFX_DEBUG_WAVES"]}


def main():
    out = os.path.join(_build.LIBDIR, "diag")
    os.makedirs(out, exist_ok=True)
    for name, defs in DIAG.items():
        p = _build.build_variant("diag_" + name, defs)
        dst = os.path.join(out, f"librfx_{name}.so")
        shutil.move(p, dst)
        print("built", dst)


if __name__ == "__main__":
    main()
