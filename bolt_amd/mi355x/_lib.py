"""ctypes binding of libbolt_mi355x.so (include/bolt_mi355x.h).

This is the binding a bolt maintainer adds next to bolt/spark (see
INTEGRATION.md).  The library is built in-tree by ``__graft_entry__.build()``
(bolt_amd/csrc/Makefile).  There is no fallback: if the library cannot be
loaded every device operation raises.
"""
import ctypes
import os

ABI_VERSION = 1

BM_BOOL, BM_U8, BM_I8, BM_U16, BM_I16, BM_U32, BM_I32, BM_U64, BM_I64, BM_F16, BM_F32, BM_F64 = range(12)
STAT_MEAN, STAT_VAR, STAT_STD, STAT_SUM, STAT_MAX, STAT_MIN = range(6)
# reduce(func) with numpy ufuncs (include/bolt_mi355x.h BM_STAT_PROD..BM_STAT_FMIN)
STAT_PROD, STAT_LAND, STAT_LOR, STAT_BAND, STAT_BOR, STAT_BXOR, STAT_FMAX, STAT_FMIN = range(6, 14)
MAX_COMBINE_PARTS = 256  # bm_reduce_combine's nparts limit (ranks of one merge)

LIB_PATH = os.environ.get("BOLT_AMD_LIB") or os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "libbolt_mi355x.so")  # env: A/B builds

# every symbol include/bolt_mi355x.h declares: name -> (restype, argtypes)
_c = ctypes
_i64p = _c.POINTER(_c.c_int64)
SIGNATURES = {
    "bm_abi_version": (_c.c_int, []),
    "bm_last_error": (_c.c_char_p, []),
    "bm_device_cus": (_c.c_int, []),
    "bm_host_writable": (_c.c_int, [_c.c_void_p, _c.c_size_t, _c.POINTER(_c.c_int)]),
    "bm_copy_strided": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _i64p, _i64p, _i64p,
                                   _c.c_int, _c.c_void_p]),
    "bm_permute": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int, _i64p,
                              _c.POINTER(_c.c_int32), _c.c_int, _c.c_void_p]),
    "bm_gather_rows": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64,
                                  _c.c_void_p, _c.c_int64, _c.c_void_p]),
    "bm_record_gather": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64,
                                    _c.c_void_p, _c.c_int, _i64p, _c.c_int, _c.c_void_p]),
    "bm_record_gather_masked": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64,
                                           _c.c_void_p, _c.c_int, _i64p, _c.c_void_p, _c.c_int, _c.c_int,
                                           _c.c_void_p]),
    "bm_record_scatter": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64,
                                     _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_int, _c.c_int, _c.c_void_p]),
    "bm_record_runs": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_int64, _c.c_int64, _c.c_int64,
                                  _c.c_int, _c.c_void_p, _c.c_int, _c.c_int, _c.c_int, _c.c_void_p]),
    "bm_reduce_workspace_bytes": (_c.c_int, [_c.c_int, _c.c_int, _c.c_int64, _c.c_int64,
                                             _c.c_int64, _c.POINTER(_c.c_size_t)]),
    "bm_reduce": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int64, _c.c_int64, _c.c_int64,
                             _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    "bm_reduce_rows": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int64, _c.c_int64, _c.c_int64,
                                  _c.c_void_p, _c.c_int, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    "bm_reduce_state_bytes": (_c.c_int, [_c.c_int, _c.c_int, _c.c_int64, _c.POINTER(_c.c_size_t)]),
    "bm_reduce_state": (_c.c_int, [_c.c_int, _c.c_void_p, _c.c_int, _c.c_int64, _c.c_int64,
                                   _c.c_int64, _c.c_void_p, _c.c_void_p, _c.c_size_t, _c.c_void_p]),
    "bm_reduce_combine": (_c.c_int, [_c.c_int, _c.c_int, _c.c_void_p, _i64p, _c.c_int, _c.c_int64,
                                     _c.c_void_p, _c.c_int, _c.c_void_p]),
    "bm_comm_unique_id": (_c.c_int, [_c.c_void_p, _c.c_size_t]),
    "bm_comm_init": (_c.c_int, [_c.POINTER(_c.c_void_p), _c.c_int, _c.c_void_p, _c.c_int]),
    "bm_comm_destroy": (_c.c_int, [_c.c_void_p]),
    "bm_comm_info": (_c.c_int, [_c.c_void_p, _c.POINTER(_c.c_int), _c.POINTER(_c.c_int), _c.c_char_p,
                                _c.c_size_t]),
    "bm_alltoallv": (_c.c_int, [_c.c_void_p, _c.c_void_p, _i64p, _i64p, _c.c_void_p, _i64p, _i64p,
                                _c.c_void_p]),
    "bm_allgatherv": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_int64, _c.c_void_p, _i64p, _i64p,
                                 _c.c_void_p]),
    "bm_comm_wait": (_c.c_int, [_c.c_void_p, _c.c_void_p, _c.c_double]),
    "bm_comm_check": (_c.c_int, [_c.c_void_p]),
    "bm_comm_abort": (_c.c_int, [_c.c_void_p]),
}
COMM_ID_BYTES = 128  # BM_COMM_ID_BYTES
RUNS_TILED = 1  # BM_RUNS_TILED
BM_OK, BM_E_ARG, BM_E_HIP, BM_E_WS, BM_E_COMM = 0, -1, -2, -3, -4

_LIB = None


class BoltDeviceError(RuntimeError):
    """A libbolt_mi355x call returned an error status."""


class BoltCommError(BoltDeviceError):
    """The RCCL communicator failed (asynchronous error, timeout, abort): a
    peer rank died, stalled or posted a mismatched exchange.  The communicator
    is aborted; the arrays of its context cannot exchange records any more."""


def load(path=LIB_PATH):
    """Load (once) and type the library; raise if it is missing or mismatched."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise BoltDeviceError(
            "libbolt_mi355x.so not found at %s: build it with `python -c \"import "
            "__graft_entry__ as g; g.build()\"` (bolt_amd/csrc/Makefile)" % path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.bm_abi_version()
    if v != ABI_VERSION:
        raise BoltDeviceError("libbolt_mi355x ABI %d, expected %d" % (v, ABI_VERSION))
    _LIB = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = _LIB.bm_last_error().decode("utf-8", "replace") if _LIB is not None else ""
        err = BoltCommError if rc == BM_E_COMM else BoltDeviceError
        raise err("%s failed (%d): %s" % (what, rc, msg))


def i64_array(vals):
    vals = [int(v) for v in vals]
    return (ctypes.c_int64 * max(1, len(vals)))(*vals)


def i32_array(vals):
    vals = [int(v) for v in vals]
    return (ctypes.c_int32 * max(1, len(vals)))(*vals)
