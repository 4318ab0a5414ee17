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

plus pip-level invariants: a stored checksum makes the packet verify, and
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
