"""The staging copies' persistent host thread pool (csrc/lsmck_pool.h): a
stress test under ThreadSanitizer (host code only; g++)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_pool_tsan(tmp_path):
    exe = tmp_path / "pool"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread",
                    "-I" + os.path.join(ROOT, "lsm_storage_engine_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "test_pool.cpp"), "-o", str(exe), "-lpthread"],
                   check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "pool ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr
