"""bench.py's launch handling (CPU): which path `--gpus N` takes with and
without a launcher, and that a launcher/--gpus mismatch is an error, not a
line that reports a GPU count it did not measure."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_no_launcher_one_gpu_is_single():
    assert bench.resolve_launch(1, {}) == ("single", 1, 0, 0)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_no_launcher_many_gpus_is_inprocess(n):
    # the driver's `python3 bench.py --gpus N` with no torchrun: one process
    # drives GPUs 0..N-1 through ptg_multi
    assert bench.resolve_launch(n, {}) == ("inprocess", 1, 0, 0)
    assert bench.resolve_launch(n, {"WORLD_SIZE": ""})[0] == "inprocess"


def test_torchrun_world_matching_gpus():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.resolve_launch(8, env) == ("torchrun", 8, 3, 3)
    assert bench.resolve_launch(1, {"WORLD_SIZE": "1", "RANK": "0"}) == ("single", 1, 0, 0)


@pytest.mark.parametrize("gpus,world", [(8, 1), (1, 8), (4, 2)])
def test_world_size_mismatch_is_an_error(gpus, world):
    with pytest.raises(ValueError):
        bench.resolve_launch(gpus, {"WORLD_SIZE": str(world)})


def test_bad_gpu_count():
    with pytest.raises(ValueError):
        bench.resolve_launch(0, {})


def test_main_exits_2_on_mismatch(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "8"])
    assert e.value.code == 2


def test_main_inprocess_without_enough_gpus_exits_2(monkeypatch):
    # no GPU in this container: --gpus 8 with no launcher refuses to render
    # fewer GPUs than it would report
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("PTG_REHEARSAL", raising=False)
    if bench.torch.cuda.device_count() >= 8:
        pytest.skip("8 GPUs visible")
    with pytest.raises(SystemExit) as e:
        bench.main(["--gpus", "8"])
    assert e.value.code == 2


def test_frame_config_defaults():
    # one frame for every N: a scaling run's lines compare
    # the metric's own box 1920x1080x1024spp frame
    a = bench.parse_args([])
    for n in (1, 2, 4, 8):
        assert bench.frame_config(a, n) == ("bench", "box", 1920, 1080, 256, 2, 1024)
    a = bench.parse_args(["--workload", "c4"])
    assert bench.frame_config(a, 8) == ("c4", "box", 3840, 2160, 1024, 2, 4096)
    a = bench.parse_args(["--workload", "c5"])
    assert bench.frame_config(a, 8)[:4] == ("c5", "synthetic:10000", 1920, 1080)


def test_metric_names_the_rendered_frame():
    assert bench.metric_of("box", 1920, 1080, 1024) == bench.METRIC
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert bench.METRIC == __import__("json").load(f)["metric"]
    m = bench.metric_of("box", 3840, 2160, 4096)
    assert m != bench.METRIC and "3840×2160×4096spp" in m and "box" in m
    assert "1920×1080×1024spp" in bench.metric_of("box_mirror", 1920, 1080, 1024)
    assert bench.metric_of("box_mirror", 1920, 1080, 1024) != bench.METRIC


def test_group_check():
    ok = bench.check_group(4, [4, 4, 4, 4], [0, 1, 2, 3], ["a", "b", "c", "d"], False)
    assert ok == []
    assert bench.check_group(4, [1, 1, 1, 1], [0, 1, 2, 3], ["a", "b", "c", "d"], False)  # 4 one-rank comms
    assert bench.check_group(4, [4, 4, 4, 4], [0, 0, 1, 1], ["a", "a", "b", "b"], False)  # shared devices
    assert bench.check_group(2, [2, 2], [0, 1], ["a", "a"], False)  # one bus id twice
    # not determinable (None) is not evidence either way; rehearsals exempt
    assert bench.check_group(2, [None, None], [0, 1], ["a", "b"], False) == []
    assert bench.check_group(4, [], [0, 0, 0, 0], ["a"] * 4, True) == []
    assert bench.check_group(1, [1], [0], ["a"], False) == []
    # unreadable bus ids (None) are not evidence either way
    assert bench.check_group(4, [4, 4, 4, 4], [0, 1, 2, 3], [None] * 4, False) == []
    assert bench.check_group(2, [2, 2], [None, None], [None, None], False) == []
    assert bench.check_group(3, [3, 3, 3], [0, 1, 2], ["a", None, "a"], False) == []


def test_launch_inprocess_flag():
    assert bench.parse_args(["--launch", "inprocess"]).launch == "inprocess"
    assert bench.parse_args([]).launch == "auto"


def test_roofline_fields():
    pmc = {"valu_fp32_share": 0.49, "hbm_bytes_per_launch": 1, "tag": "x"}
    s_bar, r = bench.roofline(100, 1200, 8 * 1200, 0, 100, 1e-6, 8, pmc)
    assert abs(s_bar - 12.0) < 1e-12
    assert r["valu_fp32_share"] == 0.49
    assert abs(r["frac_nonpacked"] / r["frac"] - bench.PEAK_FP32_TFLOPS / bench.PEAK_FP32_NONPACKED_TFLOPS) < 1e-3


def test_roofline_model_and_executed_counts():
    """The line's roofline fields say what they count:
    linear scenes price SURVEY 8(d)'s model (N tests per segment) in `frac`
    and the tests the kernel executed in `frac_executed`; BVH scenes have
    one count for both."""
    frame = 1000
    # linear, 8 spheres: 12 segments per sample, 4 tests executed per segment, 1 of them a wall
    s_bar, r = bench.roofline(frame, 12 * frame, 48 * frame, 12 * frame, 2 * 10**9, 100.0, 8, {})
    assert s_bar == 12
    assert r["model_sphere_tests_per_segment"] == 8.0
    assert r["sphere_tests_per_segment_executed"] == 4.0
    assert r["wall_tests_per_segment_executed"] == 1.0
    assert r["flop_per_sample"] == 23 * 96 + 100 * 12 + 60
    assert r["flop_per_sample_executed"] == 23 * 48 + 100 * 12 + 60
    assert r["frac_executed"] < r["frac"]
    # BVH: executed sphere and box tests are the model
    _, b = bench.roofline(frame, 2 * frame, 20 * frame, 50 * frame, 2 * 10**9, 100.0, 10000, {})
    assert b["frac"] == b["frac_executed"] and b["box_tests_per_segment"] == 25.0
    assert "wall_tests_per_segment_executed" not in b


def test_roofline_profile_provenance():
    """PMC-derived fields are copied from a committed profile: the line names
    its tag, commit and kernel-source hash, and warns when the hash is not
    this tree's kernel."""
    here = bench.ptgpu.kernel_source_hash()
    pmc = {"tag": "t", "commit": "abc1234", "kernel_hash": here, "valu_fp32_share": 0.5,
           "hbm_bytes_per_launch": 1, "valu_issue_pct": 80.0}
    _, r = bench.roofline(1000, 12000, 48000, 12000, 1000, 1.0, 8, pmc)
    assert r["profile"] == "t" and r["profile_head"] == "abc1234" and r["profile_kernel_hash"] == here
    assert "profile_warning" not in r
    _, r = bench.roofline(1000, 12000, 48000, 12000, 1000, 1.0, 8, dict(pmc, kernel_hash="000000000000"))
    assert "profile_warning" in r and "not this tree's kernel" in r["profile_warning"]


def test_committed_profiles_match_the_kernel():
    """profiles/pmc_traffic.json (what the bench line copies) was taken on
    this tree's kernel sources."""
    import json
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        recs = json.load(f)
    here = bench.ptgpu.kernel_source_hash()
    for wl in ("box 1920x1080 1024spp", "box_mirror 1920x1080 1024spp", "synthetic:10000 1920x1080 1024spp"):
        assert recs[wl]["kernel_hash"] == here, (wl, recs[wl].get("tag"))


def test_scan_kernel_name():
    assert bench.scan_kernel_name({"bvh": 1, "box_mode": 0}) == "bvh"
    assert bench.scan_kernel_name({"bvh": 0, "box_mode": 1}) == "linear, box mode"
    assert bench.scan_kernel_name({"bvh": 0, "box_mode": 0}) == "linear"
