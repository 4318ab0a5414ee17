"""Property-based checks (hypothesis) of the arithmetic every kernel relies on.

CPU only.  Three independent statements are compared on random inputs:

* ``py_standard`` -- a literal Python restatement of pip's loop
  (pip/pip_checksum.cpp:13-33: big-endian byte pairs into a u32 that wraps,
  odd tail byte << 8, two end-around folds);
* the C oracle (oracle/pipck_oracle.c, pinned to pip's compiled code by
  tests/golden);
* ``order_free`` -- the kernels' method (pip_amd/csrc/pipck_device.hpp):
  little-endian dwords of 16-byte-aligned chunks summed in any order into a
  u64, bytes outside the segment masked, one byte swap for a segment that
  starts at an even address, residue-and-zero-preserving folds.

and ``hdr_row_emulation`` -- the IPv4-header row kernel's split of each
20/24-byte item over two lanes (pip_amd/csrc/pipck_hdr.hip) -- against pip's
ip checksum; plus pip-level invariants: a stored checksum makes the packet verify, and
RFC 1624's incremental update equals recomputation except at the 0x0000 /
0xFFFF corner the kernel settles by rescanning.
"""
from __future__ import annotations

import random

import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

MASK32 = 0xFFFFFFFF


def fold(x: int) -> int:  # pip_fold_uint32, pip/pip_checksum.cpp:9-11
    return (x & 0xFFFF) + (x >> 16)


def py_standard(data: bytes, s: int = 0) -> int:
    """pip_standard_checksum (pip/pip_checksum.cpp:13-33), u32 arithmetic."""
    n = len(data)
    for i in range(0, n - 1, 2):
        s = (s + ((data[i] << 8) | data[i + 1])) & MASK32
    if n & 1:
        s = (s + (data[n - 1] << 8)) & MASK32
    return fold(fold(s))


def py_ip(data: bytes) -> int:  # pip_ip_checksum, :35-39
    return ~py_standard(data) & 0xFFFF


def py_inet(data: bytes, proto: int, src: bytes, dst: bytes) -> int:
    """pip_inet_checksum (:42-61); src/dst in network byte order, len = len(data) as u16."""
    s = 0
    for a in (src, dst):
        w = int.from_bytes(a, "big")
        s += (w >> 16) + (w & 0xFFFF)
    s += proto + (len(data) & 0xFFFF)
    return ~py_standard(data, s & MASK32) & 0xFFFF


def order_free_le_residue(mem: bytes, off: int, length: int, order_seed: int) -> int:
    """The kernels' segment sum: aligned 16-B chunks of `mem` covering
    [off, off+length), bytes outside masked, LE dwords added in a shuffled
    order into a u64, folded to 16 bits."""
    if length == 0:
        return 0
    base = off & ~15
    end = off + length
    dwords = []
    for c in range(base, end, 16):
        chunk = bytearray(mem[c:c + 16].ljust(16, b"\0"))
        for b in range(16):
            if not off <= c + b < end:
                chunk[b] = 0
        dwords += [int.from_bytes(chunk[4 * k:4 * k + 4], "little") for k in range(4)]
    random.Random(order_seed).shuffle(dwords)
    acc = sum(dwords) & ((1 << 64) - 1)
    # fold64 then fold16 (pipck_device.hpp)
    x = (acc & 0xFFFF) + ((acc >> 16) & 0xFFFF) + ((acc >> 32) & 0xFFFF) + (acc >> 48)
    return fold(fold(x))


def be_fold(le_residue: int, addr: int) -> int:
    """pipck_device.hpp be_fold: byte-swap the folded LE sum for an even start address."""
    w = fold(fold(le_residue))
    return w if addr & 1 else ((w & 0xFF) << 8) | (w >> 8)


payload = st.binary(min_size=0, max_size=3000)


@settings(max_examples=300, deadline=None)
@given(data=payload, init=st.integers(0, MASK32))
def test_oracle_equals_literal_restatement(oracle, data, init):
    assert oracle.standard_checksum(data, len(data), init) == py_standard(data, init)


@settings(max_examples=300, deadline=None)
@given(pad=st.binary(min_size=0, max_size=40), data=st.binary(min_size=0, max_size=3000),
       order_seed=st.integers(0, 2**32))
def test_order_free_kernel_sum_equals_pips_loop(pad, data, order_seed):
    """Any start offset, any summation order: the kernels' method reproduces
    pip's folded sum for segments up to 65,535 bytes (no u32 wrap)."""
    mem = pad + data + bytes(16)
    got = be_fold(order_free_le_residue(mem, len(pad), len(data), order_seed), len(pad))
    assert got == py_standard(data)


@settings(max_examples=200, deadline=None)
@given(segs=st.lists(st.binary(min_size=0, max_size=600), min_size=1, max_size=5),
       proto=st.sampled_from([6, 17]), src=st.binary(min_size=4, max_size=4),
       dst=st.binary(min_size=4, max_size=4))
def test_chain_restarts_pairing_per_segment(oracle, segs, proto, src, dst):
    """pip_inet_checksum_buf (pip_checksum.cpp:90-115): every segment is summed
    from its own start; the result equals summing the segments' folds."""
    s = 0
    for a in (src, dst):
        w = int.from_bytes(a, "big")
        s += (w >> 16) + (w & 0xFFFF)
    total = sum(len(x) for x in segs)
    s += proto + (total >> 16) + (total & 0xFFFF)
    for x in segs:
        s = py_standard(x, s)
    want = ~s & 0xFFFF
    got = oracle.inet_checksum_chain(segs, proto, src, dst)  # network-order bytes, as in_addr holds them
    assert got == want


@settings(max_examples=300, deadline=None)
@given(data=st.binary(min_size=20, max_size=2000), proto=st.sampled_from([6, 17]),
       src=st.binary(min_size=4, max_size=4), dst=st.binary(min_size=4, max_size=4))
def test_stored_checksum_verifies(data, proto, src, dst):
    """RX verification: with htons(checksum) stored in the
    (zeroed) field at offset 16, the packet sums to 0xFFFF, i.e. recomputes to 0."""
    pkt = bytearray(data)
    pkt[16:18] = b"\0\0"
    ck = py_inet(bytes(pkt), proto, src, dst)
    pkt[16:18] = ck.to_bytes(2, "big")
    assert py_inet(bytes(pkt), proto, src, dst) == 0


@settings(max_examples=300, deadline=None)
@given(data=st.binary(min_size=20, max_size=1500), new=st.binary(min_size=4, max_size=4),
       proto=st.sampled_from([6, 17]), src=st.binary(min_size=4, max_size=4),
       dst=st.binary(min_size=4, max_size=4))
def test_rfc1624_update_equals_recompute(data, new, proto, src, dst):
    """f4 (pipck_update_fixed): HC' = ~(~HC + ~m + m') over the edited words
    equals pip's recomputation whenever its folded result is not 0 -- the one
    corner (0x0000 vs 0xFFFF) the kernel settles by rescanning the packet."""
    pkt = bytearray(data)
    pkt[16:18] = b"\0\0"
    hc = py_inet(bytes(pkt), proto, src, dst)
    old = bytes(pkt[0:4])
    pkt[0:4] = new
    want = py_inet(bytes(pkt), proto, src, dst)
    s = (~hc & 0xFFFF)
    for k in (0, 2):
        m = int.from_bytes(old[k:k + 2], "big")
        m2 = int.from_bytes(new[k:k + 2], "big")
        s += (~m & 0xFFFF) + m2
    res = fold(fold(s))
    upd = ~res & 0xFFFF
    if res not in (0, 0xFFFF):
        assert upd == want
    else:  # pip gives 0x0000 for a nonzero sum and 0xFFFF for an all-zero one
        assert want in (0x0000, 0xFFFF)


def hdr_row_emulation(mem: bytes, D: int, length: int, n: int) -> list[int]:
    """k_hdr's method (pip_amd/csrc/pipck_hdr.hip) restated per lane: rows of
    C = 60 (D = 5) or 63 (D = 6) 16-byte chunks hold whole 4*D-byte items; lane l
    splits its chunk's dwords into H (the item begun in an earlier lane) and T
    (the item beginning in it) with bytes past `length` masked; the lane holding
    an item's last dword finishes it from T of the lane before plus its own H.
    dot4 = lo16 + hi16 of every masked dword (v_dot2_u32_u16 against (1, 1))."""
    C = 60 if D == 5 else 63
    PR = C * 4 // D
    masks_h, masks_t, fin = [], [], []
    for lane in range(64):
        h, t, start, f = [0] * 4, [0] * 4, 4, -1
        for i in range(4):
            d = 4 * lane + i
            q = d % D
            if q == 0 and start == 4:
                start = i
            if q == D - 1:
                f = d // D
            vb = length - 4 * q
            m = 0xFFFFFFFF if vb >= 4 else (0 if vb <= 0 else (0xFFFFFFFF >> (32 - 8 * vb)))
            h[i], t[i] = (m, 0) if i < start else (0, m)
        if lane >= C:
            h, t, f = [0] * 4, [0] * 4, -1
        masks_h.append(h), masks_t.append(t), fin.append(f)
    out = [None] * n
    rows = (n + PR - 1) // PR
    for r in range(rows):
        T = [0] * 64
        H = [0] * 64
        for lane in range(C):
            off = 16 * (C * r + lane)
            dw = [int.from_bytes(mem[off + 4 * i:off + 4 * i + 4].ljust(4, b"\0"), "little") for i in range(4)]
            H[lane] = sum((x & m & 0xFFFF) + ((x & m) >> 16) for x, m in zip(dw, masks_h[lane]))
            T[lane] = sum((x & m & 0xFFFF) + ((x & m) >> 16) for x, m in zip(dw, masks_t[lane]))
        for lane in range(64):
            hi = r * PR + fin[lane]
            if fin[lane] >= 0 and hi < n:
                s = (T[lane - 1] if lane else 0) + H[lane]
                w = fold(fold(s))
                out[hi] = ~(((w & 0xFF) << 8) | (w >> 8)) & 0xFFFF  # even starts: byte swap, then pip's ~
    return out


@settings(max_examples=60, deadline=None)
@given(stride=st.sampled_from([20, 24]), data=st.data(), n=st.integers(1, 130))
def test_header_row_split_equals_pips_ip_checksum(stride, data, n):
    """Every item of a packed 20/24-byte batch, split over two lanes as k_hdr
    splits it, gets pip_ip_checksum of its first `length` bytes."""
    length = data.draw(st.integers(0, stride))
    mem = data.draw(st.binary(min_size=n * stride, max_size=n * stride)) + bytes(1024)
    got = hdr_row_emulation(mem, stride // 4, length, n)
    assert got == [py_ip(mem[i * stride:i * stride + length]) for i in range(n)]
