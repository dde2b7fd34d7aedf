import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cpu-path-tracing_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def _ensure_oracle():
    so = os.path.join(ROOT, "oracle", "libpt_oracle.so")
    src = os.path.join(ROOT, "oracle", "pt_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "libpt_oracle.so"])


_ensure_oracle()


@pytest.fixture(scope="session")
def golden():
    out = {}
    for name in ("box", "box_mirror", "simple"):
        with open(os.path.join(GOLDEN, f"ref_{name}.json")) as f:
            out[name] = json.load(f)
    return out
