#!/usr/bin/env python3
"""Build librfx.so as of a git revision into reflaxman_amd/lib/variants/librfx_<name>.so (CPU; hipcc only), so that
tools/ab.py can time a change that no -D define switches (the current sources against an earlier commit's) in one
process.

    python tools/build_rev.py REV NAME        # e.g. python tools/build_rev.py HEAD~1 prev
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from reflaxman_amd import _build  # noqa: E402


def main():
    rev, name = sys.argv[1], sys.argv[2]
    with tempfile.TemporaryDirectory() as tmp:
        # the revision's device/host sources and the C-ABI header, laid out as in the tree
        arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "reflaxman_amd/csrc", "include"], check=True,
                              capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
        srcs = sorted(f for f in os.listdir(os.path.join(tmp, "reflaxman_amd", "csrc")) if f.endswith((".hip", ".cpp")))
        old_csrc, old_sources = _build.CSRC, _build.SOURCES
        _build.CSRC, _build.SOURCES = os.path.join(tmp, "reflaxman_amd", "csrc"), srcs
        try:
            out = os.path.join(_build.LIBDIR, "variants", f"librfx_{name}.so")
            os.makedirs(os.path.dirname(out), exist_ok=True)
            _build._compile_link(out, [], os.path.join(tmp, "obj"))
        finally:
            _build.CSRC, _build.SOURCES = old_csrc, old_sources
    print("built", out)


if __name__ == "__main__":
    main()
