"""bench.py helpers that need no GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_strong_scaling_baseline_is_the_committed_one_gpu_c4_line():
    b = bench.one_gpu_line("c4", 7680, 4320, 8)
    assert b is not None and b["unit"] == "Mrays/s" and b["value"] > 0
    assert b["source"].startswith("profiles" + os.sep) and os.sep + "configs" + os.sep in b["source"]
    assert bench.one_gpu_line("c4", 640, 360, 8) is None  # another frame: no baseline


def test_default_one_gpu_line_times_the_c4_denominator():
    """The driver's N = 1 line (default config C3) carries c4_1gpu, the C4 frame every N > 1 line renders, timed on one
    GPU in the same run; other configs, custom frames and --no-c4 do not."""
    assert bench.times_c4_denominator(1, "c3", False, False)
    assert not bench.times_c4_denominator(1, "c3", False, True)
    assert not bench.times_c4_denominator(1, "c3", True, False)
    assert not bench.times_c4_denominator(2, "c4", False, False)
    assert not bench.times_c4_denominator(1, "c5", False, False)
    ap_default = bench.CONFIGS["c4"]
    assert ap_default[:4] == ("synth16", 7680, 4320, 8) and bench.CONFIGS["c3"][0] == ap_default[0]


def test_cpu_sample_strides_cover_every_config():
    """Every config has a bounded CPU sample: a row stride (one-sample frames) or a band of rows (SSAA frames)."""
    one = {k for k, c in bench.CONFIGS.items() if c[4] == 1}
    assert set(bench.CPU_STRIDE) == one
    assert set(bench.CPU_BAND_ROWS) == set(bench.CONFIGS) - one


def test_weak_and_strong_frame_sizes():
    assert bench.frame_size(1, 3840, 2160, "weak") == (3840, 2160)
    assert bench.frame_size(8, 7680, 4320, "strong") == (7680, 4320)
    w, h = bench.frame_size(4, 3840, 2160, "weak")
    assert (w, h) == (7680, 4320)


def test_roofline_frac_is_a_hardware_fraction():
    """roofline.frac is the executed VALU lane-op fraction (<= 1) from a PMC record, or null without one; the
    reference-equivalent rate (above the peak on C5) lives in effective_ref_flops."""
    import glob
    import json
    from reflaxman_amd import metrics
    recs = [json.load(open(p)) for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc", "*.json")))]
    assert recs
    for rec in recs:
        # the record's own kernel time: GRBM_GUI_ACTIVE is summed over the 8 XCDs, at 2.4 GHz
        ms = rec["counters"]["GRBM_GUI_ACTIVE"] / 8 / 2.4e6
        ex = metrics.executed_work(rec, ms)
        r = metrics.roofline(ex, rec.get("hbm_bytes_per_launch"), 5e12, ms, 8294400)
        assert 0 < r["frac"] <= 1 and r["achieved"] <= r["peak"], (rec.get("config"), ms, r["frac"])
        assert r["unit"] == "T VALU lane-op/s" and r["peak"] == 78.6
    r = metrics.roofline(None, None, 9e12, 3.35, 8294400)  # C5-like effective work: above the peak ...
    assert r["frac"] is None and r["effective_ref_flops"]["frac"] > 1  # ... but never as `frac`


def test_no_committed_line_has_frac_above_one():
    """Every bench line committed under profiles/ carries a hardware fraction (or null) in roofline.frac."""
    import glob
    import json
    seen = 0
    for p in glob.glob(os.path.join(ROOT, "profiles", "**", "*.json"), recursive=True):
        text = open(p).read()
        for chunk in [text] + text.splitlines():
            try:
                d = json.loads(chunk)
            except ValueError:
                continue
            if isinstance(d, dict) and isinstance(d.get("roofline"), dict):
                seen += 1
                f = d["roofline"].get("frac")
                assert f is None or 0 <= f <= 1, (p, f)
    assert seen > 0


def test_gpus_n_without_launcher_starts_the_ranks(monkeypatch):
    """`bench.py --gpus N` (N > 1) with no WORLD_SIZE runs N ranks as a torch.distributed.run child job (rendezvous on
    127.0.0.1, the same arguments) and returns its exit code -- it never measures one GPU and calls it N."""
    import subprocess
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.setattr(subprocess, "run", fake_run)
    argv = ["--gpus", "2", "--steps", "3", "--one-device", "--backend", "gloo"]
    assert bench.main(argv) == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-len(argv) - 1:] == [os.path.abspath(bench.__file__)] + argv
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and 0 < int(port[0].split("=")[1]) < 65536


def test_gpus_must_match_the_launchers_world(monkeypatch):
    """Under a launcher, --gpus must equal WORLD_SIZE: a mismatch exits 2 before anything is measured."""
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "4"]) == 2
