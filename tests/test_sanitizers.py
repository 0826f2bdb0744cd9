"""Host ASan + UBSan run ("Host ASan/UBSan builds of the CPU
restatement").  The reference's safety net is Zig's ReleaseSafe checks
(build.zig:12); here every host source that handles scene data (scene_io,
image_io, bvh_build, accel_build) and the oracle are built with
-fsanitize=address,undefined -fno-sanitize-recover=all and driven through the C ABI
by tools/sanitize/san_driver.cpp: scenes 0-4 loaded, BVHs built and compared with the
oracle's, the wide tree built, oracle renders in both RNG modes, closest-hit
queries, binary scene and PNG round trips, and the error paths (unknown scene,
missing / truncated files).  Any report, leak included, fails the run.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_host_sources_clean_under_asan_ubsan(tmp_path):
    out = str(tmp_path)
    subprocess.run(["make", "-s", "-j4", "-C", os.path.join(REPO, "tools", "sanitize"), "OUT=" + out],
                   check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(out, "san_driver"), os.path.join(REPO, "assets"), out],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitized host run ok" in r.stdout
