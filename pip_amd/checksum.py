"""pip's checksum API (pip/pip_checksum.h:17-34), one packet at a time, on the GPU.

Same names, argument meaning and results as the reference functions; byte
buffers are Python ``bytes``-like objects, addresses are 4-/16-byte network
order values (``socket.inet_pton`` output), and a ``pip_buf`` chain is a list
of segments.  Every call goes through ``pipck_host_sum`` (pip's exact
per-segment semantics, u32 wrap included, computed by a HIP kernel); there is
no host compute path.  For throughput use :mod:`pip_amd.engine` batches.
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Sequence

from ._lib import HSeg, call, load

_tls = threading.local()


def _ctx() -> C.c_void_p:
    ctx = getattr(_tls, "ctx", None)
    if ctx is None:
        ctx = C.c_void_p()
        call("pipck_ctx_create", -1, C.byref(ctx))
        _tls.ctx = ctx
    return ctx


def set_zero_copy(mode: int) -> None:
    """This thread's per-packet path: 0 staged, 1 zero-copy, 2 auto, 3 resident, 4 resident with a device-memory
    doorbell (pipck_ctx_zero_copy)."""
    call("pipck_ctx_zero_copy", _ctx(), mode)


def _device_sum(segments: Sequence[bytes], init: int) -> int:
    bufs = [C.create_string_buffer(bytes(s), max(len(s), 1)) for s in segments]
    arr = (HSeg * max(len(segments), 1))()
    for i, (s, b) in enumerate(zip(segments, bufs)):
        arr[i].ptr = C.cast(b, C.c_void_p)
        arr[i].len = len(s)
    out = C.c_uint32(0)
    call("pipck_host_sum", _ctx(), arr, len(segments), init & 0xFFFFFFFF, C.byref(out))
    return out.value


def _split(a: int) -> int:
    return (a >> 16) + (a & 0xFFFF)


def _addr_terms(addr: bytes) -> int:
    return sum(_split(int.from_bytes(addr[i:i + 4], "big")) for i in range(0, len(addr), 4))


def pip_fold_uint32(num: int) -> int:
    """pip/pip_checksum.cpp:9-11."""
    num &= 0xFFFFFFFF
    return (num & 0xFFFF) + (num >> 16)


def pip_standard_checksum(payload: bytes, length: int | None = None, sum: int = 0) -> int:  # noqa: A002
    """pip/pip_checksum.cpp:13-33 (``length`` defaults to ``len(payload)``)."""
    n = len(payload) if length is None else length
    return _device_sum([bytes(payload[:n])], sum)


def pip_ip_checksum(payload: bytes, length: int | None = None) -> int:
    """pip/pip_checksum.cpp:35-39."""
    return ~pip_standard_checksum(payload, length, 0) & 0xFFFF


def pip_inet_checksum(payload: bytes, proto: int, src: bytes, dst: bytes, length: int | None = None) -> int:
    """pip/pip_checksum.cpp:42-61; ``length`` is a u16 as in pip."""
    n = (len(payload) if length is None else length) & 0xFFFF
    pseudo = _addr_terms(src) + _addr_terms(dst) + (proto & 0xFF) + n
    return ~pip_standard_checksum(payload, n, pseudo) & 0xFFFF


def pip_inet6_checksum(payload: bytes, proto: int, src: bytes, dst: bytes, length: int | None = None) -> int:
    """pip/pip_checksum.cpp:63-87."""
    return pip_inet_checksum(payload, proto, src, dst, length)


def pip_inet_checksum_buf(chain: Sequence[bytes], proto: int, src: bytes, dst: bytes) -> int:
    """pip/pip_checksum.cpp:90-115: per-segment sums over a pip_buf chain."""
    total = sum(len(s) for s in chain) & 0xFFFFFFFF
    pseudo = _addr_terms(src) + _addr_terms(dst) + (proto & 0xFF) + _split(total)
    return ~_device_sum(list(chain), pseudo) & 0xFFFF


def pip_inet6_checksum_buf(chain: Sequence[bytes], proto: int, src: bytes, dst: bytes) -> int:
    """pip/pip_checksum.cpp:118-148."""
    return pip_inet_checksum_buf(chain, proto, src, dst)


__all__ = ["pip_fold_uint32", "pip_standard_checksum", "pip_ip_checksum", "pip_inet_checksum",
           "pip_inet6_checksum", "pip_inet_checksum_buf", "pip_inet6_checksum_buf", "load"]
