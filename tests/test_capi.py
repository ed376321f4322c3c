"""The C-ABI library loads on a GPU-less host and exports every function
include/pmdfc_cceh.h declares (no compute calls here)."""
import os
import re
import subprocess

import pytest

from conftest import REPO


def _declared(header="pmdfc_cceh.h"):
    src = open(os.path.join(REPO, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pmdfc_[a-z0-9_]+)\s*\(", src)))


def test_header_declarations_match_python_binding():
    from pmdfc_amd.engine import EXPORTS
    assert sorted(EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    from pmdfc_amd.engine import LIB_PATH, load_library
    L = load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in _declared() if s not in syms]
    assert not missing, missing
    for s in _declared():
        assert getattr(L, s) is not None


def test_kv_header_matches_binding_and_library():
    """include/pmdfc_kv.h (the per-op front-end) against pmdfc_amd.kv and
    libpmdfc_gpucceh.so."""
    from pmdfc_amd.kv import KV_EXPORTS, KV_LIB_PATH, load_kv_library
    assert sorted(KV_EXPORTS) == _declared("pmdfc_kv.h")
    L = load_kv_library()
    out = subprocess.run(["nm", "-D", "--defined-only", KV_LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in KV_EXPORTS if s not in syms]
    assert not missing, missing
    for s in KV_EXPORTS:
        assert getattr(L, s) is not None


def test_host_only_entry_points():
    from pmdfc_amd import depth_for_hybrid, depth_for_src, load_library
    L = load_library()
    assert L.pmdfc_abi_version() == 8
    # test_KV: KV(10 GiB*10/4096) -> src CCEH(26214400) -> depth 14
    assert depth_for_src(26214400) == 14
    assert depth_for_hybrid(16384) == 14
    assert depth_for_hybrid(65536) == 16
    assert depth_for_hybrid(2) == 1


def test_no_cpu_fallback():
    """The product path fails loudly without a GPU instead of computing on CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from pmdfc_amd import CCEH, PmdfcError
    with pytest.raises(PmdfcError):
        CCEH(2)


def test_product_package_never_imports_oracle():
    pat = re.compile(r"(import\s+oracle|from\s+oracle|liboracle|\boc_[a-z_]+\()")
    pkg = os.path.join(REPO, "pmdfc_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(root, f)).read()
                assert not pat.search(txt), f
