"""pytest configuration.

Markers:
  gpu — needs an MI355X; run with ``pytest -m gpu`` on the GPU box.  Every
        other test runs on CPU (``-m "not gpu"``) and never launches a kernel.
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _ensure_built():
    lib = os.path.join(REPO, "zraytrace_amd", "libzrt.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(REPO, "zraytrace_amd", "csrc")], check=True)
    # the oracle is rebuilt whenever it is older than its sources or include/zrt.h
    # (a stale build would read zrt_stats with an old layout); a second of gcc
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(REPO, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def scenes():
    import zraytrace_amd as z
    cache = {}

    def get(i):
        if i not in cache:
            cache[i] = z.load_scene(i)
        return cache[i]
    return get
