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
@pytest.mark.parametrize("world,partition", [(2, "bands"), (3, "bands"), (2, "strips"), (3, "strips")])
def test_bench_multirank_frame_matches_single_gpu(world, partition):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--width", "640", "--height", "360",
           "--backend", "gloo", "--one-device", "--no-cpu-baseline", "--partition", partition]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == world
    assert out["parity"]["multi_rank_frame_equals_single_gpu"] is True
    # the step after the timed ones, down the steady-state path (look-aheads on: gloo ranks on one GPU stage their
    # all-gathers through host memory on the side stream), equals a single-GPU render of the same stream frame
    assert out["steady_state_parity"]["equals_single_gpu"] is True
    assert "count-ahead" in out["config"]["parallelism"] and "emit-ahead" in out["config"]["parallelism"]
    b = out["strong_scaling_baseline"]
    assert b["value"] > 0 and b["efficiency"] > 0
    assert out["roofline"]["frac"] is None or out["roofline"]["frac"] <= 1
    assert out["value"] > 0
    if partition == "bands":
        b = out["band_bounds"]
        assert len(b) == world + 1 and b[0] == 0 and b[-1] == 360


def _count_ahead_worker(emit_ahead):
    """Rank 0 of 1 over RCCL: StripFrame with count-ahead (the next frame's RNG count and its all-gather on a side
    stream after the emit event) -- and with emit-ahead, the next frame's emit there too, into the second randDir
    buffer -- over 6 frames, against the same frames from rfx_render_frame."""
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from reflaxman_amd import scenes
    from reflaxman_amd.dist import RfxStripOps, StripFrame
    from reflaxman_amd.render import Renderer, build_scene, make_frame

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        scene, cam = build_scene(scenes.get_scene("synth16"))
        W, H, D, seed = 640, 360, 8, 1350490027
        stream = torch.cuda.Stream(device=dev)
        torch.cuda.set_stream(stream)
        ra, rb = Renderer(device=0, sphere_seed=seed), Renderer(device=0, sphere_seed=seed)
        for r in (ra, rb):
            r.set_scene(scene)
            r.set_stream(stream.cuda_stream)
        sf = StripFrame(RfxStripOps(ra, make_frame(cam, W, H, D, 1), stream.cuda_stream), W, H, 8, 0, 1, dev,
                        count_ahead=True, emit_ahead=emit_ahead)
        assert sf.count_ahead and sf.ahead is None and sf.emit_ahead == emit_ahead
        fb = make_frame(cam, W, H, D, 1)
        img = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
        argb = torch.zeros(H * W, dtype=torch.int32, device=dev)
        ok = []
        for i in range(6):
            if i == 4:
                sf.drop_lookahead()  # frame 4 counts afresh on the main stream
            out = sf.step().clone()
            rb.render_frame(fb, img.data_ptr(), argb.data_ptr(), 0, stream.cuda_stream)
            ok.append(bool(torch.equal(out.reshape(-1), argb)) and bool(torch.equal(sf.img[: H * W * 3], img)))
        torch.cuda.synchronize()
        print(json.dumps({"frames_equal": ok}))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("emit_ahead", [0, 1])
def test_count_ahead_rccl_frames_equal_plain_frames(emit_ahead):
    env = {**os.environ, "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_port())}
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "count_ahead", str(emit_ahead)], capture_output=True,
                       text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["frames_equal"] == [True] * 6, out


if __name__ == "__main__" and sys.argv[1:2] == ["count_ahead"]:
    _count_ahead_worker(bool(int(sys.argv[2])))
