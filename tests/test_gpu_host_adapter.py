"""The drop-in C++ IHash backend (pmdfc_amd/host/gpu_cceh.*) under the
reference harness pattern: concurrent per-op Insert/Get from 8 threads through
the MPSC batching front-end (tests/cpp/test_gpu_kv.cpp)."""
import os
import subprocess

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_gpu_kv_harness_zero_failed_search():
    exe = os.path.join(REPO, "pmdfc_amd", "lib", "test_gpu_kv")
    r = subprocess.run([exe, "200000", "8"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failedSearch" in r.stdout
    assert "false_hits 0" in r.stdout
    assert "bf_negatives 0" in r.stdout  # the attached counting BF saw every Insert
    assert "extent_bad 0" in r.stdout  # ICCEH adapter: hybrid extents
