"""The C-ABI library loads and exports every symbol include/rpc_hip.h declares (CPU only:
no compute call is made without a GPU)."""
import os
import re

from robustpointclouds_amd import _ffi
from tests.conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "rpc_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rpc_\w+)\s*\(", txt, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert "rpc_hard_voxelize" in names and "rpc_perturber_backward" in names


def test_library_exports_every_declared_symbol():
    lib = _ffi.load()
    for name in _declared():
        assert hasattr(lib, name), name
        assert name in _ffi.SIGNATURES, f"{name} has no ctypes signature"
    assert b"gfx950" in lib.rpc_version()
