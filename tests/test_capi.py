"""CPU-side checks of the C-ABI boundary: the library loads (no GPU needed),
exports every symbol include/slam_hip.h declares, and the ctypes structs match
the C struct sizes."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "slam_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(slam_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "slam_pf_step" in names and "slam_pf_create" in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from slamhip import _lib
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) <= set(_lib.SIGNATURES)


def test_version_and_device_query_without_gpu():
    from slamhip import _lib
    lib = _lib.load()
    assert lib.slam_version() >= 10000
    n = ctypes.c_int(-1)
    assert lib.slam_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


def test_struct_layouts():
    from slamhip import _lib
    assert ctypes.sizeof(_lib.PFConfig) == 8 * (1 + 1 + 4 + 9 + 6 + 3 + 1) + 8
    assert ctypes.sizeof(_lib.PFResult) == 8 * (3 + 9 + 3 + 1) + 24


def test_create_without_device_fails_loudly():
    from slamhip import _lib
    from slamhip.pf import DeviceParticleFilter
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.SlamError):
        DeviceParticleFilter(100, [[0.0, 0.0]])


def test_graph_record_layouts_match_the_c_structs():
    """slam_graph_edge (4 int64 + 6 double) and slam_graph_half (3 int64 + 3
    double) as the NumPy record types the bindings pass through ctypes."""
    from slamhip.graph import EDGE_DTYPE, HALF_DTYPE
    assert EDGE_DTYPE.itemsize == 80 and HALF_DTYPE.itemsize == 48
    assert [HALF_DTYPE.fields[f][1] for f in ("time", "pose", "landmark", "obs")] == [0, 8, 16, 24]
