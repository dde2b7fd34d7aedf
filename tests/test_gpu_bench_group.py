"""bench.py's proof of the RCCL group behind an N-GPU line (VERDICT r4 next
1), on the 1-GPU box: the one-process path's communicators
(ptg_multi_comm_info) and the torchrun path's (the default process group's
RCCL communicator read with torch's own librccl) both report a one-rank group
on device 0 here; the 8-GPU node reports 8."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROBE = r"""
import os, sys, json
sys.path.insert(0, os.environ["ROOT"])
import bench, torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1)
dist.barrier()
cnt, dev, ur, why = bench.torch_rccl_info(0)
print(json.dumps({"count": cnt, "device": dev, "user_rank": ur, "why": why, "bus": bench.bus_id_of(0)}))
dist.destroy_process_group()
"""


def _require_gpu():
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need a visible MI355X")


def test_torch_process_group_rccl_info():
    _require_gpu()
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT="29517")
    out = subprocess.run([sys.executable, "-c", _PROBE], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert (rec["count"], rec["device"], rec["user_rank"]) == (1, 0, 0), rec
    assert rec["bus"] and ":" in rec["bus"]


def test_bench_inprocess_line_carries_the_group():
    """--launch inprocess at --gpus 1: a one-rank ncclCommInitAll group; the
    line names the metric's frame and carries rccl_ranks and the bus id."""
    _require_gpu()
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--launch", "inprocess", "--gpus", "1",
                          "--steps", "1", "--warmup", "1", "--t1", "off", "--width", "256", "--height", "128",
                          "--spp", "16"], capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["rccl_ranks"] == [1] and line["launch"] == "inprocess"
    assert line["devices"][0]["device"] == 0 and ":" in line["devices"][0]["pci_bus_id"]
    assert line["group_check"].startswith("ok")
    assert line["config"]["workload"] == "box 256x128 16spp" and "256×128×16spp" in line["metric"]
