"""pipck_rx_verify (include/pipck.h, pip_amd/csrc/pipck_rx.hip) through its C
ABI with ctypes: the RX batch verifier behind pip_checksum_amd_verify_packets
(SURVEY.md 8 f2), checked against packets whose checksums the oracle (pip's
arithmetic, pip/pip_checksum.cpp:35-87) filled in.  The drop-in's own tests
(tests/test_boundary.py) run the same kernel through the shim."""
import ctypes as C
import random

import numpy as np
import pytest

from tests.test_boundary import IP_OK, L4_CHECKED, UNCHECKED, VERIFIED, _ext, _rx_packet


def _rxq():
    from pip_amd import _lib

    lib = _lib.load()
    q = C.c_void_p()
    assert lib.pipck_rxq_create(None, C.byref(q)) == 0
    return lib, q


def _run(lib, q, ptrs, lens):
    n = len(ptrs)
    arr = (C.c_void_p * max(n, 1))(*ptrs)
    ln = (C.c_uint32 * max(n, 1))(*lens)
    ok = np.full(max(n, 1), 0xEE, dtype=np.uint8)
    good = C.c_uint64(12345)
    rc = lib.pipck_rx_verify(q, arr, ln, n, ok.ctypes.data, C.byref(good))
    assert rc == 0, lib.pipck_last_error()
    assert good.value == int((ok[:n] == VERIFIED).sum())
    return ok[:n]


@pytest.mark.gpu
def test_rx_verify_c_abi_chunks_jumbo_and_staging(oracle):
    """More packets than one kernel launch takes (2,048), lengths up to 64 KB
    (many rows per wave), heap packets that grow the staging copy in the middle
    of a call, pinned packets at odd addresses read in place, and damage in the
    header, the payload or the checksum field -- each caught in its own bit."""
    from pip_amd import _lib

    rng = random.Random(101)
    pkts, want = [], []
    for k in range(5000):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        l4len = rng.choice([rng.randint(20, 1500), rng.randint(8000, 9000), rng.randint(60000, 65400)]) \
            if k % 50 == 0 else rng.randint(20, 1500)
        p = bytearray(_rx_packet(oracle, rng, fam, proto, l4len, k + 1))
        checked = not (fam == 4 and proto == 17 and (k + 1) % 7 == 0)
        w = VERIFIED if checked else UNCHECKED
        r = k % 4
        hl = 20 if fam == 4 else 40
        if r == 1 and checked:
            i = rng.randrange(hl, len(p))
            if fam == 4 and proto == 17 and i in (hl + 6, hl + 7):
                i = hl  # not the UDP checksum field: a zero there would mean "no checksum"
            p[i] ^= 0x08  # any other L4 byte
            w = IP_OK | L4_CHECKED
        elif r == 2 and fam == 4:
            p[rng.choice([1, 4, 5, 8, 10, 11])] ^= 0x40  # an IPv4 header byte only its own checksum covers
            w &= ~IP_OK
        pkts.append(bytes(p) + rng.randbytes(rng.choice([0, 3])))  # link padding after the IP length
        want.append(w)
    lib, q = _rxq()
    try:
        heap = [C.create_string_buffer(p, len(p)) for p in pkts]
        ok = _run(lib, q, [C.cast(h, C.c_void_p).value for h in heap], [len(p) for p in pkts])
        assert list(ok) == want
        # the same packets in a pinned ring, every other one, at odd addresses
        size = sum(len(p) + 8 for p in pkts) + 64
        base = lib.pipck_host_alloc(size)
        assert base
        try:
            ptrs, off = [], 5
            for i, p in enumerate(pkts):
                C.memmove(base + off, p, len(p))
                ptrs.append(base + off if i % 2 == 0 else C.cast(heap[i], C.c_void_p).value)
                off += len(p) + (i % 8)
            ok2 = _run(lib, q, ptrs, [len(p) for p in pkts])
            assert list(ok2) == want
        finally:
            assert lib.pipck_host_free(C.c_void_p(base)) == 0  # the call released its holds
    finally:
        lib.pipck_rxq_destroy(q)
    assert (np.array(want) == VERIFIED).sum() > 1000


@pytest.mark.gpu
def test_rx_verify_c_abi_edges(oracle):
    """Empty batches, null packets and junk, IPv6 extension-header walks, and
    the C ABI's argument errors."""
    from pip_amd import _lib

    rng = random.Random(3)
    lib, q = _rxq()
    try:
        assert _run(lib, q, [], []).size == 0
        cases = [(b"", 0), (bytes(19), 0), (bytes([0x45]) + bytes(30), 0),
                 (_rx_packet(oracle, rng, 6, 6, 200, 1, ext=_ext([(0, 0), (60, 1)], 6)), VERIFIED),
                 (_rx_packet(oracle, rng, 6, 17, 200, 2, ext=_ext([(44, 0x0001)], 17)), UNCHECKED),
                 (_rx_packet(oracle, rng, 4, 6, 40, 3, frag=0x2000), UNCHECKED),
                 (_rx_packet(oracle, rng, 4, 1, 8, 4), VERIFIED)]
        bufs = [C.create_string_buffer(p, max(len(p), 1)) for p, _ in cases]
        ptrs = [C.cast(b, C.c_void_p).value for b in bufs]
        ptrs[0] = None  # a null packet pointer: ok 0
        ok = _run(lib, q, ptrs, [len(p) for p, _ in cases])
        assert list(ok) == [w for _, w in cases]
        ok8 = np.zeros(1, dtype=np.uint8)
        assert lib.pipck_rx_verify(None, None, None, 1, ok8.ctypes.data, None) == _lib.PIPCK_EINVAL
        assert lib.pipck_rx_verify(q, None, None, 1, ok8.ctypes.data, None) == _lib.PIPCK_EINVAL
    finally:
        lib.pipck_rxq_destroy(q)
