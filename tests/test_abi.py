"""The C-ABI library: builds, loads without a GPU, exports every symbol that
include/shockwave_amd.h declares, and fails loudly (no CPU fallback) when no
GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

import sw_native as sn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shockwave_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sw_[a-z_]+)\s*\(", src)))


def test_header_declares_the_python_symbol_list():
    assert sorted(sn.EXPORTED_SYMBOLS) == declared_functions()


def test_library_exports_every_declared_symbol():
    assert os.path.exists(sn.LIB_PATH), "run __graft_entry__.build() first"
    out = subprocess.check_output(["nm", "-D", "--defined-only", sn.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in declared_functions() if s not in exported]
    assert not missing, missing


def test_library_loads_and_reports_version():
    lib = sn.load()
    assert lib.sw_abi_version() == 2


def test_structs_match_header_layout():
    # sizes of the C structs on x86-64 (pointers 8 B, natural alignment)
    assert ctypes.sizeof(sn.SwProblem) == 4 * 4 + 8 * 2 + 8 * 8
    assert ctypes.sizeof(sn.SwResult) == 8 * 2 + 8 * 5 + 4 * 2 + 8
    assert ctypes.sizeof(sn.SwConfig) == 4 * 2 + 8 + 4 + 4 + 8


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(sn.NativeError):
        sn.Solver(device=0)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(sn.NativeError):
        sn.load(str(tmp_path / "nope.so"))
