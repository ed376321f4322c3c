"""Build-container checks of the drop-in boundary against the reference's own
headers and front-ends (skipped where /root/reference is absent, e.g. on the
GPU box).  Compiles, with the reference's include path first:

* GpuCCEH : IHash against server/IHash.h, GpuCCEHHybrid : ICCEH against
  server/ICCEH.h -- each in its own translation unit (the two headers share
  the include guard HASH_INTERFACE_H_);
* server/KV.cpp with integration/KV.cpp.gpucceh.patch and -DGPUCCEH;
* server/NuMA_KV.cpp with integration/NuMA_KV.cpp.gpucceh.patch;
* the linked harnesses of oracle/Makefile `dropin` (test_KV, replay_KV,
  NUMA_KV driver) into a temporary directory.
No GPU call happens here; tests/test_gpu_dropin.py runs the binaries."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

SERVER = "/root/reference/server"
pytestmark = pytest.mark.skipif(not os.path.isdir(SERVER), reason="reference tree absent")
HOST = os.path.join(REPO, "pmdfc_amd", "host")


def _cxx(tmp_path, src_text, name, extra=()):
    src = tmp_path / f"{name}.cpp"
    src.write_text(src_text)
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-DPMDFC_REFERENCE_HEADERS", f"-I{SERVER}", f"-I{HOST}",
           *extra, str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


def test_ihash_facade_compiles_against_reference_ihash(tmp_path):
    _cxx(tmp_path, "#include <cstdint>\n#include <vector>\n"  # as KV.h does before IHash.h
         '#include "IHash.h"\n#include "gpu_cceh.h"\n'
         "IHash* make() { return new pmdfc_host::GpuCCEH(26214400); }\n", "ihash")


def test_iccehfacade_compiles_against_reference_icceh(tmp_path):
    _cxx(tmp_path, "#include <cstdint>\n#include <vector>\n"  # as NuMA_KV.h does before ICCEH.h
         '#include "ICCEH.h"\n#include "gpu_cceh_hybrid.h"\n'
         "ICCEH* make() { return new pmdfc_host::GpuCCEHHybrid(16384); }\n", "icceh")


def test_icceh_facade_with_numa_kv_header(tmp_path):
    """NuMA_KV.h pulls ICCEH.h and CCEH_hybrid.h; the facade must coexist."""
    _cxx(tmp_path, '#include "NuMA_KV.h"\n#include "gpu_cceh_hybrid.h"\n'
         "ICCEH* make() { return new pmdfc_host::GpuCCEHHybrid(16384); }\n", "numakv")


def test_patches_apply_and_build_the_reference_front_ends(tmp_path):
    """oracle/Makefile dropin: the reference's KV.cpp / NuMA_KV.cpp patched by
    integration/*.patch, with test_KV.cpp / replay_KV.cpp / our NUMA_KV
    driver, linked against libpmdfc_gpucceh.so."""
    lib = os.path.join(REPO, "pmdfc_amd", "lib", "libpmdfc_gpucceh.so")
    if not os.path.exists(lib):
        pytest.skip("libpmdfc_gpucceh.so not built")
    work = tmp_path / "oracle"
    shutil.copytree(os.path.join(REPO, "oracle"), work, ignore=shutil.ignore_patterns("_ref", "*.so", "__pycache__"))
    os.symlink(os.path.join(REPO, "integration"), tmp_path / "integration")
    os.symlink(os.path.join(REPO, "pmdfc_amd"), tmp_path / "pmdfc_amd")
    r = subprocess.run(["make", "-s", "-C", str(work), "dropin", f"PATCHED={tmp_path / 'patched'}"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    for b in ("julee_kv_gpu", "replay_kv_gpu", "numa_kv_gpu"):
        assert os.access(work / "_ref" / b, os.X_OK), b
    # the patches touch only the backend switch / the ctor (maintainer-sized)
    for p in ("KV.cpp.gpucceh.patch", "NuMA_KV.cpp.gpucceh.patch"):
        txt = open(os.path.join(REPO, "integration", p)).read()
        added = [l for l in txt.splitlines() if l.startswith("+") and not l.startswith("+++")]
        assert 0 < len(added) <= 12, p
