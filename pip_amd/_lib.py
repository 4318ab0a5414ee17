"""ctypes binding of libpipck.so (the C ABI declared in include/pipck.h).

The library is built in-tree by ``pip_amd/Makefile`` (``__graft_entry__.build()``).
There is no fallback: if the shared object is missing, importing the engine
raises, so a GPU run can never silently take another path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "lib"
# PIPCK_LIB points a process at another build of the same ABI (tools/ab_scan.py
# runs each build in its own process: two builds in one process would share
# kernel symbol names, and the HIP runtime would launch one build's kernels
# for both).
LIBPIPCK = Path(os.environ.get("PIPCK_LIB") or LIB_DIR / "libpipck.so")
LIBSHIM = LIB_DIR / "libpip_checksum_amd.so"

PIPCK_OK, PIPCK_EINVAL, PIPCK_ERANGE, PIPCK_EHIP, PIPCK_ENODEV, PIPCK_ENOMEM, PIPCK_EBUSY = range(7)
MAX_SEG_LEN = 65535
HDR_NONE, HDR_TCP, HDR_UDP, HDR_IPV4 = 0, 1, 2, 3

_u8, _u16, _u32, _u64, _i32 = C.c_uint8, C.c_uint16, C.c_uint32, C.c_uint64, C.c_int
_p, _sz = C.c_void_p, C.c_size_t


class Flow4(C.Structure):
    _fields_ = [("src", _u32), ("dst", _u32), ("proto", _u8), ("pad", _u8 * 3)]


class Flow6(C.Structure):
    _fields_ = [("src", _u8 * 16), ("dst", _u8 * 16), ("proto", _u8), ("pad", _u8 * 3)]


class Desc(C.Structure):
    _fields_ = [("offset", _u64), ("len", _u32), ("flow", _u32)]


class HSeg(C.Structure):
    _fields_ = [("ptr", _p), ("len", _u32)]


# name -> (restype, argtypes); must match include/pipck.h (checked by tests/test_abi.py)
SIGNATURES = {
    "pipck_last_error": (C.c_char_p, []),
    "pipck_version": (_u32, []),
    "pipck_flows4_prepare": (_i32, [_p, _u32, _p, _p]),
    "pipck_flows6_prepare": (_i32, [_p, _u32, _p, _p]),
    "pipck_checksum_fixed": (_i32, [_p, _u64, _u32, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_checksum_ragged": (_i32, [_p, _p, _u64, _p, _p, _p, _p]),
    "pipck_checksum_packed": (_i32, [_p, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_verify_packed": (_i32, [_p, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_packed_index": (_i32, [_p, _u64, _p, _p]),
    "pipck_checksum_packed_bytes": (_i32, [_p, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_host_checksum_packed_bytes": (_i32, [_p, _p, _p, _u64, _i32, _p, _u32, _u64, _p]),
    "pipck_checksum_packed_n": (_i32, [_p, _u64, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_verify_packed_n": (_i32, [_p, _u64, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_checksum_packed_bytes_n": (_i32, [_p, _u64, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_verify_packed_bytes_n": (_i32, [_p, _u64, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_verify_packed_bytes": (_i32, [_p, _p, _p, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_packed_bytes_index": (_i32, [_p, _u64, _p, _p]),
    "pipck_gen_packed_bytes": (_i32, [_p, _p, _p, _u64, _u64, _u64, _u32, _p]),
    "pipck_checksum_chains": (_i32, [_p, _p, _u64, _p, _p, _u64, _p, _p, _p, _p, _p]),
    "pipck_verify_fixed": (_i32, [_p, _u64, _u32, _u64, _p, _u32, _p, _u64, _p, _p]),
    "pipck_verify_ragged": (_i32, [_p, _p, _u64, _p, _p, _p, _p]),
    "pipck_update_fixed": (_i32, [_p, _u64, _u64, _u32, _u32, _u32, _u32, _u32, _p, _u64, _p, _p, _u32, _p, _u64,
                                  _p]),
    "pipck_cfg_seed": (_u64, [_u32]),
    "pipck_gen_fixed": (_i32, [_p, _u64, _u32, _u64, _u64, _u64, _u32, _p]),
    "pipck_gen_zipf_lengths": (_i32, [_p, _u64, _u64, _u64, _p]),
    "pipck_gen_ragged_layout": (_i32, [_p, _u64, _u64, _u32, _p, C.POINTER(_u64), _p]),
    "pipck_gen_ragged_fill": (_i32, [_p, _p, _u64, _u64, _u64, _u32, _p]),
    "pipck_gen_flows4": (_i32, [_p, _u32, _u64, _u8, _p]),
    "pipck_gen_flows6": (_i32, [_p, _u32, _u64, _u8, _p]),
    "pipck_ctx_create": (_i32, [_i32, C.POINTER(_p)]),
    "pipck_ctx_destroy": (_i32, [_p]),
    "pipck_host_sum": (_i32, [_p, C.POINTER(HSeg), _u32, _u32, C.POINTER(_u32)]),
    "pipck_host_checksum_fixed": (_i32, [_p, _p, _u64, _u32, _u64, _i32, _p, _u32, _u64, _p]),
    "pipck_host_alloc": (_p, [_sz]),
    "pipck_host_free": (_i32, [_p]),
    "pipck_txq_create": (_i32, [_p, C.POINTER(_p)]),
    "pipck_txq_destroy": (_i32, [_p]),
    "pipck_txq_add4": (_i32, [_p, C.POINTER(HSeg), _u32, _u8, _u32, _u32, _p]),
    "pipck_txq_add6": (_i32, [_p, C.POINTER(HSeg), _u32, _u8, _p, _p, _p]),
    "pipck_txq_add_ip": (_i32, [_p, _p, _u32, _p]),
    "pipck_txq_add4_zc": (_i32, [_p, C.POINTER(HSeg), _u32, _u8, _u32, _u32, _p]),
    "pipck_txq_add6_zc": (_i32, [_p, C.POINTER(HSeg), _u32, _u8, _p, _p, _p]),
    "pipck_host_register": (_i32, [_p, _sz]),
    "pipck_host_unregister": (_i32, [_p]),
    "pipck_txq_pending": (_u64, [_p]),
    "pipck_txq_flush": (_i32, [_p]),
    "pipck_ctx_zero_copy": (_i32, [_p, _i32]),
    "pipck_txq_submit": (_i32, [_p]),
    "pipck_txq_complete": (_i32, [_p]),
    "pipck_txq_inflight": (_u64, [_p]),
    "pipck_txq_auto_zero_copy": (_i32, [_p, _i32]),
    "pipck_txq_inplace_max": (_i32, [_p, _u64]),
    "pipck_rxq_create": (_i32, [_p, C.POINTER(_p)]),
    "pipck_rxq_destroy": (_i32, [_p]),
    "pipck_rx_verify": (_i32, [_p, _p, _p, _u64, _p, C.POINTER(_u64)]),
    "pipck_rx_verify_device": (_i32, [_p, _u64, _p, _p, _u64, _p, _p, _p]),
    "pipck_host_rx_verify_packed": (_i32, [_p, _p, _p, _u64, _p, C.POINTER(_u64)]),
    "pipck_rx_verify_ring": (_i32, [_p, _u64, _p, _u64, _p, _p]),
    "pipck_rx_verify_ring_n": (_i32, [_p, _u64, _p, _u64, _p, _p, _p]),
    "pipck_checksum_ragged_n": (_i32, [_p, _u64, _p, _u64, _p, _u32, _p, _p, _p]),
    "pipck_verify_ragged_n": (_i32, [_p, _u64, _p, _u64, _p, _u32, _p, _p, _p]),
    "pipck_checksum_chains_n": (_i32, [_p, _u64, _p, _u64, _p, _p, _u64, _p, _u32, _p, _p, _p, _p]),
    "pipck_checksum_fixed_n": (_i32, [_p, _u64, _u32, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_verify_fixed_n": (_i32, [_p, _u64, _u32, _u64, _p, _u32, _p, _u64, _p, _p, _p]),
    "pipck_update_fixed_n": (_i32, [_p, _u64, _u64, _u32, _u32, _u32, _u32, _u32, _p, _u64, _p, _p, _u32, _p, _u64,
                                    _p, _p]),
}

# the internal tuning hook (pip_amd/csrc/pipck_testing.h): tests and tools only
INTERNAL_SIGNATURES = {
    "pipck_tune": (None, [_u32, _u32, _u32, _u32]),
    "pipck_tune_probes": (None, [_u32]),
    "pipck_tune_ring": (None, [_u32]),
    "pipck_trace_tasks": (_i32, [_p, _u64]),
    "pipck_tune_xcd_weights": (_i32, [_p, _u32]),
    "pipck_last_launch": (_i32, [C.c_char_p, _sz]),
}

_lib = None


class PipckError(RuntimeError):
    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} -> status {rc}: {msg}")
        self.rc = rc


def load() -> C.CDLL:
    """Load libpipck.so once; raise if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIBPIPCK.exists():
        raise RuntimeError(
            f"{LIBPIPCK} is missing: build it with `make -C {LIB_DIR.parent}` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(os.fspath(LIBPIPCK), mode=C.RTLD_GLOBAL)
    for name, (res, args) in {**SIGNATURES, **INTERNAL_SIGNATURES}.items():
        if os.environ.get("PIPCK_LIB") and not hasattr(lib, name):
            continue  # an older build under A/B may predate some entry points
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(fn: str, rc: int) -> None:
    if rc != PIPCK_OK:
        msg = load().pipck_last_error()
        raise PipckError(fn, rc, msg.decode() if msg else "")


def call(fn: str, *args) -> None:
    check(fn, getattr(load(), fn)(*args))
