"""ASan + UBSan build of the host engine (sanitizers on host
code), driven by tests/cpu_selftest.cpp against the C oracle on random
workloads (ingest in chunks, quantiles, merge folds; eps 0.2 .. 0.001)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpu_engine_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "sketches-py_amd", "cpu"), "sanitize"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "cpu_selftest: ok" in r.stdout
