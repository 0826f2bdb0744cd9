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


def _lib_source_id(lib):
    """The source half of the built library's zrt_build_id(), read in a child
    process (this one must not map a library that make may replace)."""
    code = ("import ctypes, sys; f = ctypes.CDLL(sys.argv[1]).zrt_build_id; f.restype = ctypes.c_char_p; "
            "print(f().decode())")
    r = subprocess.run([sys.executable, "-c", code, lib], capture_output=True, text=True)
    return r.stdout.strip().split("-")[0] if r.returncode == 0 else None


def _ensure_built():
    lib = os.path.join(REPO, "zraytrace_amd", "libzrt.so")
    csrc = os.path.join(REPO, "zraytrace_amd", "csrc")
    from zraytrace_amd import build_id_of_sources
    want = build_id_of_sources()
    # (ZRT_LIB: the tests run an A/B build variant; the in-tree library is left as
    # it is - rebuilding it from the tree's sources here would make a later A/B
    # run of "the shipped library" in the same session the variant too)
    if not os.environ.get("ZRT_LIB") and (not os.path.exists(lib) or _lib_source_id(lib) != want):
        # missing, or stale against its sources: rebuild, and
        # refuse to test a library that still does not match the tree
        subprocess.run(["make", "-s", "-j8", "-C", csrc], check=True)
        got = _lib_source_id(lib)
        if got != want:
            raise RuntimeError(f"libzrt.so build id {got} does not match its sources {want} after a rebuild")
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
