"""The C-ABI library loads and exports every entry point include/bolt_mi355x.h
declares, with the documented argument checking (no GPU needed: these calls
fail before touching a device)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "bolt_mi355x.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bm_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from bolt_amd.mi355x import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libbolt_mi355x.so is not built (run __graft_entry__.build())")
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    from bolt_amd.mi355x import _lib
    names = header_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    assert sorted(_lib.SIGNATURES) == names  # the ctypes binding covers exactly the header


def test_abi_version(lib):
    from bolt_amd.mi355x import _lib
    assert lib.bm_abi_version() == _lib.ABI_VERSION == 1


def test_argument_errors(lib):
    from bolt_amd.mi355x import _lib
    rc = lib.bm_copy_strided(None, None, -1, None, None, None, 4, None)
    assert rc == -1 and b"bad arguments" in lib.bm_last_error()
    rc = lib.bm_permute(None, None, 2, _lib.i64_array([2, 3]), _lib.i32_array([0, 0]), 4, None)
    assert rc == -1 and b"invalid permutation" in lib.bm_last_error()
    n = ctypes.c_size_t(0)
    assert lib.bm_reduce_workspace_bytes(0, 10, 1, 0, 5, ctypes.byref(n)) == -1
    assert b"empty reduction" in lib.bm_last_error()
    assert lib.bm_reduce(7, None, 10, 1, 1, 1, None, 10, None, 0, None) == -1
    assert lib.bm_reduce_combine(0, 10, None, None, 65, 1, None, 10, None) == -1
    assert lib.bm_gather_rows(None, None, 1, 4, 0, None, 3, None) == -1
    assert b"bad sizes" in lib.bm_last_error()
    assert lib.bm_gather_rows(None, None, 1, 4, 8, None, 3, None) == -1
    assert b"null pointer" in lib.bm_last_error()
    assert lib.bm_gather_rows(None, None, 0, 4, 8, None, 3, None) == 0  # nothing to move
    assert lib.bm_record_gather(None, None, 4, 8, 8, None, 0, None, 16, None) == -1
    assert b"bad arguments" in lib.bm_last_error()
    assert lib.bm_record_gather(None, None, 4, 8, 8, None, 0, None, 8, None) == -1
    assert b"null pointer" in lib.bm_last_error()
    assert lib.bm_record_gather(None, None, 0, 8, 8, None, 0, None, 8, None) == 0  # nothing to move
    # parts must tile the destination record in order, sources inside the record
    assert lib.bm_record_gather(None, None, 1, 8, 8, None, 2, _lib.i64_array([0, 4, 0, 4, 5, 8, 4, 8]), 8,
                                None) == -1
    assert b"does not tile" in lib.bm_last_error()
    assert lib.bm_record_gather(None, None, 1, 8, 8, None, 2, _lib.i64_array([0, 4, 0, 4, 4, 8, 4, 9]), 8,
                                None) == -1
    assert lib.bm_record_gather(None, None, 1, 8, 8, None, 9, None, 8, None) == -1
    ok = ctypes.c_int(7)
    assert lib.bm_host_writable(None, 0, None) == -1
    assert lib.bm_host_writable(None, 16, ctypes.byref(ok)) == 0 and ok.value == 0


def test_workspace_and_state_sizes(lib):
    n = ctypes.c_size_t(0)
    # C2 mean over time on the key=time layout: [1][2000][262144] -> chunked over R
    assert lib.bm_reduce_workspace_bytes(0, 10, 1, 2000, 262144, ctypes.byref(n)) == 0
    assert n.value % (262144 * 8) == 0 and n.value > 0
    # row reduction with many rows needs no chunking
    assert lib.bm_reduce_workspace_bytes(2, 10, 262144, 2000, 1, ctypes.byref(n)) == 0
    assert n.value == 0
    assert lib.bm_reduce_state_bytes(1, 10, 100, ctypes.byref(n)) == 0 and n.value == 1600
    assert lib.bm_reduce_state_bytes(0, 3, 100, ctypes.byref(n)) == 0 and n.value == 800
    assert lib.bm_reduce_state_bytes(3, 3, 100, ctypes.byref(n)) == 0 and n.value == 800


def test_record_runs_argument_errors(lib):
    """bm_record_runs refuses bad geometry before any launch: records not a
    multiple of the group, vector widths that do not divide the record /
    stride or exceed 16 B, a tiled walk with more than 64 runs, unknown flags,
    null pointers; zero records is a no-op."""
    from bolt_amd.mi355x import _lib
    f = lib.bm_record_runs
    assert f(None, None, 6, 64, 4, 256, 2, None, 16, 0, 8, None) == -1  # 6 records, group 4
    assert b"bad arguments" in lib.bm_last_error()
    assert f(None, None, 8, 63, 4, 256, 2, None, 16, 0, 8, None) == -1  # 63 f64 not a 16-B multiple
    assert f(None, None, 8, 64, 4, 256, 2, None, 32, 0, 8, None) == -1  # 32-B vectors
    assert f(None, None, 8, 64, 4, 256, 2, None, 4, 0, 8, None) == -1   # vector narrower than an element
    assert f(None, None, 8, 64, 4, 256, 65, None, 16, _lib.RUNS_TILED, 8, None) == -1
    assert f(None, None, 8, 64, 4, 256, 2, None, 16, 2, 8, None) == -1   # unknown flag
    assert b"flags" in lib.bm_last_error()
    assert f(None, None, 8, 64, 4, 256, 2, None, 16, 0, 8, None) == -1   # null pointers
    assert b"null pointer" in lib.bm_last_error()
    assert f(None, None, 0, 64, 4, 256, 2, None, 16, _lib.RUNS_TILED, 8, None) == 0  # nothing to move
    rc = lib.bm_record_scatter(None, None, 4, 64, 4, 256, None, None, 3, 8, None)  # vec not a power of two
    assert rc == -1 and b"bad arguments" in lib.bm_last_error()
