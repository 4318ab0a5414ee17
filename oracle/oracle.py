"""TEST INFRASTRUCTURE ONLY: ctypes access to the parity oracle.

* ``Oracle``    -- oracle/_build/libpipck_oracle.so, the clean-room C restatement
                   of pip/pip_checksum.cpp plus the CPU twin of the generator.
* ``Reference`` -- oracle/_ref/libpipref.so, pip's REAL pip_checksum.cpp compiled
                   from /root/reference by ``make -C oracle ref`` (present where it
                   was built; it travels to the GPU box as a built artefact).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg use
this module, and only as the checker / the reported CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_SO = HERE / "_build" / "libpipck_oracle.so"
REF_SO = HERE / "_ref" / "libpipref.so"

_u8, _u16, _u32, _u64, _i32, _p = C.c_uint8, C.c_uint16, C.c_uint32, C.c_uint64, C.c_int, C.c_void_p
_pp = C.POINTER(C.c_void_p)


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", os.fspath(HERE)], check=True)


def _buf(data) -> tuple[C.Array, int]:
    b = bytes(data)
    return C.create_string_buffer(b, max(len(b), 1)), len(b)


def _np_ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


class _Common:
    lib: C.CDLL
    prefix: str

    def _fn(self, name):
        return getattr(self.lib, self.prefix + name)

    def fold_uint32(self, x: int) -> int:
        return self._fn("fold_uint32")(x & 0xFFFFFFFF)

    def standard_checksum(self, data, length=None, s=0) -> int:
        b, n = _buf(data)
        return self._fn("standard_checksum")(b, n if length is None else length, s & 0xFFFFFFFF)

    def ip_checksum(self, data, length=None) -> int:
        b, n = _buf(data)
        return self._fn("ip_checksum")(b, n if length is None else length)

    def inet_checksum(self, data, proto, src: bytes, dst: bytes, length=None) -> int:
        b, n = _buf(data)
        s = int.from_bytes(src, "little")  # in-memory s_addr
        d = int.from_bytes(dst, "little")
        return self._fn("inet_checksum")(b, proto, s, d, (n if length is None else length) & 0xFFFF)

    def inet6_checksum(self, data, proto, src: bytes, dst: bytes, length=None) -> int:
        b, n = _buf(data)
        return self._fn("inet6_checksum")(b, proto, bytes(src), bytes(dst), (n if length is None else length) & 0xFFFF)

    def _chain(self, segs):
        bufs = [_buf(s) for s in segs]
        ptrs = (C.c_void_p * max(len(segs), 1))(*[C.cast(b, C.c_void_p) for b, _ in bufs])
        lens = (C.c_uint32 * max(len(segs), 1))(*[n for _, n in bufs])
        return bufs, ptrs, lens

    def inet_checksum_chain(self, segs, proto, src: bytes, dst: bytes) -> int:
        keep, ptrs, lens = self._chain(segs)
        return self._fn("inet_checksum_chain")(ptrs, lens, len(segs), proto, int.from_bytes(src, "little"),
                                              int.from_bytes(dst, "little"))

    def inet6_checksum_chain(self, segs, proto, src: bytes, dst: bytes) -> int:
        keep, ptrs, lens = self._chain(segs)
        return self._fn("inet6_checksum_chain")(ptrs, lens, len(segs), proto, bytes(src), bytes(dst))


def _declare(lib, prefix):
    f = lambda n: getattr(lib, prefix + n)  # noqa: E731
    f("fold_uint32").restype = _u32
    f("fold_uint32").argtypes = [_u32]
    f("standard_checksum").restype = _u32
    f("standard_checksum").argtypes = [_p, _u32, _u32]
    f("ip_checksum").restype = _u16
    f("ip_checksum").argtypes = [_p, _u32]
    f("inet_checksum").restype = _u16
    f("inet_checksum").argtypes = [_p, _u8, _u32, _u32, _u16]
    f("inet6_checksum").restype = _u16
    f("inet6_checksum").argtypes = [_p, _u8, C.c_char_p, C.c_char_p, _u16]
    f("inet_checksum_chain").restype = _u16
    f("inet_checksum_chain").argtypes = [_pp, C.POINTER(_u32), _u32, _u8, _u32, _u32]
    f("inet6_checksum_chain").restype = _u16
    f("inet6_checksum_chain").argtypes = [_pp, C.POINTER(_u32), _u32, _u8, C.c_char_p, C.c_char_p]


class Oracle(_Common):
    prefix = "ock_"

    def __init__(self):
        if not ORACLE_SO.exists():
            build_oracle()
        self.lib = C.CDLL(os.fspath(ORACLE_SO))
        _declare(self.lib, self.prefix)
        L = self.lib
        L.ock_mix64.restype = _u64
        L.ock_mix64.argtypes = [_u64]
        L.ock_cfg_seed.restype = _u64
        L.ock_cfg_seed.argtypes = [_u32]
        L.ock_gen_packet.argtypes = [_u64, _u64, _u32, _u32, _p, _u64]
        L.ock_gen_flow4.argtypes = [_u64, _u32, C.POINTER(_u32), C.POINTER(_u32)]
        L.ock_gen_flow6.argtypes = [_u64, _u32, C.c_char_p, C.c_char_p]
        L.ock_zipf_len.restype = _u32
        L.ock_zipf_len.argtypes = [_u64, _u64]
        L.ock_batch_fixed.argtypes = [_p, _u64, _u32, _u64, _i32, _u8, _u64, _u32, _u64, _p, _i32]
        L.ock_batch_ragged.argtypes = [_p, _p, _p, _u64, _i32, _u8, _u64, _u32, _u64, _p, _i32]
        L.ock_gen_fixed_batch.argtypes = [_u64, _u64, _u64, _u32, _u32, _p, _u64, _i32]
        L.ock_gen_ragged_layout.restype = _u64
        L.ock_gen_ragged_layout.argtypes = [_u64, _u64, _u64, _p, _p]
        L.ock_gen_ragged_fill.argtypes = [_u64, _u64, _u64, _u32, _p, _p, _p, _i32]

    # ---- generator twin
    def mix64(self, x: int) -> int:
        return self.lib.ock_mix64(x & 0xFFFFFFFFFFFFFFFF)

    def packet(self, seed: int, pkt: int, length: int, hdr: int, stride: int | None = None) -> bytes:
        stride = length if stride is None else stride
        b = C.create_string_buffer(max(stride, 1))
        self.lib.ock_gen_packet(seed, pkt, length, hdr, b, stride)
        return b.raw[:stride]

    def flow4(self, seed: int, flow: int) -> tuple[bytes, bytes]:
        s, d = _u32(), _u32()
        self.lib.ock_gen_flow4(seed, flow, C.byref(s), C.byref(d))
        return s.value.to_bytes(4, "little"), d.value.to_bytes(4, "little")

    def flow6(self, seed: int, flow: int) -> tuple[bytes, bytes]:
        s, d = C.create_string_buffer(16), C.create_string_buffer(16)
        self.lib.ock_gen_flow6(seed, flow, s, d)
        return s.raw[:16], d.raw[:16]

    def flows_table(self, family: int, seed: int, n_flows: int, proto: int) -> bytes:
        """Flow records in the pipck_flow4 / pipck_flow6 layout (include/pipck.h)."""
        out = bytearray()
        for f in range(n_flows):
            if family == 4:
                s, d = self.flow4(seed, f)
                out += s + d + bytes([proto, 0, 0, 0])
            else:
                s, d = self.flow6(seed, f)
                out += s + d + bytes([proto, 0, 0, 0])
        return bytes(out)

    def zipf_len(self, seed: int, pkt: int) -> int:
        return self.lib.ock_zipf_len(seed, pkt)

    def zipf_lengths(self, seed: int, first: int, n: int) -> np.ndarray:
        return np.array([self.lib.ock_zipf_len(seed, first + i) for i in range(n)], dtype=np.uint32)

    def gen_fixed_batch(self, seed: int, first: int, n: int, length: int, hdr: int, stride: int,
                        threads: int = 1) -> np.ndarray:
        arena = np.zeros(n * stride, dtype=np.uint8)
        self.lib.ock_gen_fixed_batch(seed, first, n, length, hdr, _np_ptr(arena), stride, threads)
        return arena

    def gen_ragged_batch(self, seed: int, first: int, n: int, hdr: int, threads: int = 1):
        """Zipf batch in the device layout (offsets = prefix of lengths rounded to 16):
        (arena, offsets, lens)."""
        lens = np.zeros(max(n, 1), dtype=np.uint32)
        offs = np.zeros(max(n, 1), dtype=np.uint64)
        total = self.lib.ock_gen_ragged_layout(seed, first, n, _np_ptr(lens), _np_ptr(offs))
        arena = np.zeros(max(int(total), 16), dtype=np.uint8)
        self.lib.ock_gen_ragged_fill(seed, first, n, hdr, _np_ptr(lens), _np_ptr(offs), _np_ptr(arena), threads)
        return arena, offs[:n], lens[:n]

    def gen_packed_bytes_batch(self, seed: int, first: int, n: int, hdr: int):
        """Zipf batch in the byte-packed layout (no padding between packets): (arena, offsets, lens).
        Same packet bytes as gen_ragged_batch; packets filled in order on one thread, so each packet's
        16-byte-rounded zero tail is overwritten by the next packet."""
        lens = np.zeros(max(n, 1), dtype=np.uint32)
        offs16 = np.zeros(max(n, 1), dtype=np.uint64)
        self.lib.ock_gen_ragged_layout(seed, first, n, _np_ptr(lens), _np_ptr(offs16))
        lens = lens[:n]
        offs = np.zeros(max(n, 1), dtype=np.uint64)
        if n:
            offs[1:n] = np.cumsum(lens[:-1], dtype=np.uint64)
        total = int(offs[n - 1] + lens[n - 1]) if n else 0
        arena = np.zeros(total + 32, dtype=np.uint8)
        self.lib.ock_gen_ragged_fill(seed, first, n, hdr, _np_ptr(lens), _np_ptr(offs), _np_ptr(arena), 1)
        arena[total:] = 0
        return arena[:(total + 15) // 16 * 16], offs[:n], lens

    # ---- batch checksums
    def batch_fixed(self, arena: np.ndarray, stride: int, length: int, n: int, family: int, proto: int,
                    seed: int, n_flows: int, flow_origin: int = 0, threads: int = 1) -> np.ndarray:
        out = np.zeros(n, dtype=np.uint16)
        self.lib.ock_batch_fixed(_np_ptr(arena), stride, length, n, family, proto, seed, n_flows, flow_origin,
                                 _np_ptr(out), threads)
        return out

    def batch_ragged(self, arena: np.ndarray, offsets: np.ndarray, lens: np.ndarray, family: int, proto: int,
                     seed: int, n_flows: int, flow_origin: int = 0, threads: int = 1) -> np.ndarray:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros(len(lens), dtype=np.uint16)
        self.lib.ock_batch_ragged(_np_ptr(arena), _np_ptr(offsets), _np_ptr(lens), len(lens), family, proto, seed,
                                  n_flows, flow_origin, _np_ptr(out), threads)
        return out


class Reference(_Common):
    """pip's own pip_checksum.cpp (compiled from /root/reference into oracle/_ref)."""

    prefix = "ref_"

    def __init__(self):
        if not REF_SO.exists():
            raise FileNotFoundError(f"{REF_SO} not built (make -C oracle ref, needs /root/reference)")
        self.lib = C.CDLL(os.fspath(REF_SO))
        _declare(self.lib, self.prefix)
        self.lib.ref_batch_fixed.argtypes = [_p, _u64, _u32, _u64, _i32, _u8, _p, _p, _u32, _u64, _p, _i32]
        self.lib.ref_batch_ragged.argtypes = [_p, _p, _p, _u64, _i32, _u8, _p, _p, _u32, _u64, _p, _i32]
        self.lib.ref_chains_build.argtypes = [_p, _p, _p, _u64, _u32]
        self.lib.ref_chains_build.restype = _p
        self.lib.ref_chains_free.argtypes = [_p]
        self.lib.ref_chains_checksum.argtypes = [_p, _i32, _u8, _p, _p, _u32, _u64, _p, _i32]

    @staticmethod
    def available() -> bool:
        return REF_SO.exists()

    @staticmethod
    def _flow_arrays(family: int, flows: bytes, n_flows: int):
        rec = 12 if family == 4 else 36
        raw = np.frombuffer(flows, dtype=np.uint8).reshape(n_flows, rec) if family else None
        f4 = f6 = None
        if family == 4:
            f4 = np.ascontiguousarray(raw[:, :8]).view(np.uint32).reshape(-1).copy()
        elif family == 6:
            f6 = np.ascontiguousarray(raw[:, :32]).copy()
        return f4, f6

    def batch_fixed(self, arena: np.ndarray, stride: int, length: int, n: int, family: int, proto: int,
                    flows: bytes, n_flows: int, flow_origin: int = 0, threads: int = 1) -> np.ndarray:
        """flows: pipck_flow4/6 records as produced by Oracle.flows_table."""
        out = np.zeros(n, dtype=np.uint16)
        f4, f6 = self._flow_arrays(family, flows, n_flows)
        self.lib.ref_batch_fixed(_np_ptr(arena), stride, length, n, family, proto,
                                 None if f4 is None else _np_ptr(f4), None if f6 is None else _np_ptr(f6),
                                 max(n_flows, 1), flow_origin, _np_ptr(out), threads)
        return out

    def tx_chains(self, arena: np.ndarray, offsets: np.ndarray, lens: np.ndarray, hdr_len: int) -> "RefChains":
        """Each packet as pip's TX path builds it (pip_tcp_packet.cpp:28-37): a hdr_len-byte header
        pip_buf chained to the payload pip_buf, both pointing into ``arena`` (which must outlive them)."""
        return RefChains(self, arena, offsets, lens, hdr_len)

    def batch_ragged(self, arena: np.ndarray, offsets: np.ndarray, lens: np.ndarray, family: int, proto: int,
                     flows: bytes, n_flows: int, flow_origin: int = 0, threads: int = 1) -> np.ndarray:
        """pip_inet{,6}_checksum per packet of a ragged batch (pip_checksum.cpp:42-87)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        out = np.zeros(len(lens), dtype=np.uint16)
        f4, f6 = self._flow_arrays(family, flows, n_flows)
        self.lib.ref_batch_ragged(_np_ptr(arena), _np_ptr(offsets), _np_ptr(lens), len(lens), family, proto,
                                  None if f4 is None else _np_ptr(f4), None if f6 is None else _np_ptr(f6),
                                  max(n_flows, 1), flow_origin, _np_ptr(out), threads)
        return out


class RefChains:
    """pip_buf chains built by pip's own code; ``checksum`` calls pip_inet{,6}_checksum_buf per packet
    (pip_checksum.cpp:90-148) -- the call pip_tcp_packet.cpp:124-134 makes -- on ``threads`` threads."""

    def __init__(self, ref: Reference, arena: np.ndarray, offsets: np.ndarray, lens: np.ndarray, hdr_len: int):
        self.ref = ref
        self._arena = arena
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        self.n = len(lens)
        self.h = ref.lib.ref_chains_build(_np_ptr(arena), _np_ptr(offsets), _np_ptr(lens), self.n, hdr_len)

    def checksum(self, family: int, proto: int, flows: bytes, n_flows: int, flow_origin: int = 0,
                 threads: int = 1) -> np.ndarray:
        out = np.zeros(self.n, dtype=np.uint16)
        f4, f6 = Reference._flow_arrays(family, flows, n_flows)
        self.ref.lib.ref_chains_checksum(self.h, family, proto, None if f4 is None else _np_ptr(f4),
                                         None if f6 is None else _np_ptr(f6), max(n_flows, 1), flow_origin,
                                         _np_ptr(out), threads)
        return out

    def close(self) -> None:
        if self.h:
            self.ref.lib.ref_chains_free(self.h)
            self.h = None

    def __del__(self):
        self.close()
