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
    a = bench.parse_args([])
    assert bench.frame_config(a, 1) == ("bench", "box", 1920, 1080, 256, 2, 1024)
    assert bench.frame_config(a, 8) == ("c4", "box", 3840, 2160, 1024, 2, 4096)
    a = bench.parse_args(["--workload", "c5"])
    assert bench.frame_config(a, 8)[:4] == ("c5", "synthetic:10000", 1920, 1080)
