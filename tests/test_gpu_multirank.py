"""The bench's multi-rank path end to end on one GPU: N ranks (torch.distributed.run, gloo, all on
cuda:0) run the sliced RNG pre-pass, trace their strips, gather and assemble the frame; rank 0 checks
the assembled frame against a single-GPU render of the same frame (bench.py parity field)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_bench_multirank_frame_matches_single_gpu(world):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--width", "640", "--height", "360",
           "--backend", "gloo", "--one-device", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == world
    assert out["parity"]["multi_rank_frame_equals_single_gpu"] is True
    assert out["value"] > 0
