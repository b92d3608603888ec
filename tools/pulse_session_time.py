#!/usr/bin/env python3
"""Drop-in cost per interactive frame: the reference's Pulse (unmodified, headless, tests/native/pulse_headless.cpp)
driving the drop-in Render at 640x480 through its session (still additive frames at depth 15, motion frames in
block preview at depth 4), under both renderNext policies -- "span" (each chunk rendered as Pulse asks for it:
~19 chunks per frame, doubling from 1 pixel, Pulse.cpp:125,141-142) and "frame" (the whole frame at the first
renderNext).  Runs the session `--reps` times per policy (no hashing: the time is that of Pulse's
exec() calls), interleaved, and prints one JSON line with the median ms per still and per motion frame.

    python tools/pulse_session_time.py [--reps 5] [--out profiles/r03/pulse_session_640x480.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "tests", "native", "_build", "pulse_dropin")


def session(policy: str, tick: int, W: int, H: int, tmp: str):
    env = {**os.environ, "RFX_DROPIN_POLICY": policy}
    r = subprocess.run([DROPIN, tmp + "/", "session", str(W), str(H), str(tick), "nohash"], capture_output=True,
                       text=True, env=env, timeout=300, check=True)
    return [(int(l.split()[3]), float(l.split()[5]), float(l.split()[9])) for l in r.stdout.splitlines()
            if l.startswith("frame ")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tick", type=int, default=1000)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    W, H = 640, 480
    # frame roles of the session at tick 1000 (tests/golden/manifest.json pulse_session_640x480_tick1000): 0, 1 still
    # (depth 15 additive), 2 the abandoned still frame + the first motion frame, 3..12 motion (block preview -1,
    # depth 4), 13..15 still again
    still, motion = [0, 1, 13, 14, 15], list(range(3, 13))
    res = {p: [] for p in ("span", "frame")}
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        for _ in range(args.reps):
            for p in res:
                res[p].append(session(p, args.tick, W, H, tmp))
    out = {"what": "drop-in Render under the reference's Pulse, 640x480 session (tests/native/pulse_headless.cpp), "
                   "ms of Pulse's exec() calls per completed frame; *_incl_first_read adds the window's first pixel "
                   "read (waits for the frame on the device, copies the 3.7 MB float frame to the host)",
           "tick_us": args.tick, "reps": args.reps}
    for p, runs in res.items():
        per = lambda idx, k: statistics.median(statistics.median(run[i][k] for i in idx) for run in runs)
        both = lambda idx: statistics.median(statistics.median(run[i][1] + run[i][2] for i in idx) for run in runs)
        out[p] = {"still_ms_per_frame": round(per(still, 1), 4), "motion_ms_per_frame": round(per(motion, 1), 4),
                  "still_ms_incl_first_read": round(both(still), 4), "motion_ms_incl_first_read": round(both(motion), 4),
                  "renderNext_calls_per_frame": runs[0][3][0],
                  "frames": [round(statistics.median(run[i][1] for run in runs), 4) for i in range(len(runs[0]))]}
    print(json.dumps(out))
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        open(args.out, "w").write(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
