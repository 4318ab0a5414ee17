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


# ---- pipck_rx_verify_device: the same packets already in device memory ---------


@pytest.fixture(params=[4, 2, 1])
def tile_waves(request):
    """k_packedb_rx's block width (waves streaming one tile): 4 is the default
    (a ring of 8), 2 = tune loads_per_lane 28 (a ring of 16), 1 = 32 (a ring of
    32); the test checks the launch took it."""
    from pip_amd import engine

    engine.tune(loads_per_lane={4: 0, 2: 28, 1: 32}[request.param])
    yield request.param
    engine.tune()


def _rx_kernel_waves():
    from pip_amd import _lib

    buf = C.create_string_buffer(4096)
    _lib.check("pipck_last_launch", _lib.load().pipck_last_launch(buf, len(buf)))
    name = buf.value.decode().split("(")[0]
    assert "k_packedb_rx<" in name, name
    return int(name.rsplit(",", 1)[1].rstrip("> "))
def _device_batch(frames):
    """Frames back to back in a device arena (the byte-packed layout), u16 lengths, tile index."""
    import torch

    from pip_amd import engine

    total = sum(len(f) for f in frames)
    buf = np.zeros(total + 32, dtype=np.uint8)  # readable past the last frame's 16-byte chunk
    off = 0
    for f in frames:
        buf[off:off + len(f)] = np.frombuffer(f, dtype=np.uint8)
        off += len(f)
    arena = torch.from_numpy(buf).to("cuda")
    lens = torch.from_numpy(np.array([len(f) for f in frames], dtype=np.uint16).view(np.int16)).to("cuda")
    return arena, lens, engine.packed_bytes_index(lens)


def _ipv4(oracle, proto, l4, src=b"\x0a\0\0\x01", dst=b"\x0a\0\0\x02"):
    import struct

    hdr = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + len(l4), 7, 0, 64, proto, 0, src, dst))
    c = oracle.ip_checksum(bytes(hdr))
    hdr[10:12] = struct.pack(">H", c)
    return bytes(hdr) + bytes(l4)


@pytest.mark.gpu
def test_rx_verify_device_equals_host_path(oracle, tile_waves):
    """pipck_rx_verify_device (packets in HBM, parsed on the GPU, payload sums
    derived from the k_packedb stream's frame sums) gives exactly the bits the host-parsed
    pipck_rx_verify gives, on 5,000 oracle-checksummed IPv4/IPv6
    TCP/UDP/ICMP packets up to 64 KB with damage in the header, the payload or
    the checksum field and link padding after the IP length."""
    import torch

    from pip_amd import engine

    rng = random.Random(202)
    pkts, want = [], []
    for k in range(5000):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        l4len = rng.choice([rng.randint(20, 1500), rng.randint(8000, 9000), rng.randint(60000, 65400)]) \
            if k % 50 == 0 else rng.randint(20, 1500)
        p = bytearray(_rx_packet(oracle, rng, fam, proto, l4len, k + 1))
        checked = not (fam == 4 and proto == 17 and (k + 1) % 7 == 0)
        w = VERIFIED if checked else UNCHECKED
        hl = 20 if fam == 4 else 40
        if k % 4 == 1 and checked:
            i = rng.randrange(hl, len(p))
            if fam == 4 and proto == 17 and i in (hl + 6, hl + 7):
                i = hl
            p[i] ^= 0x08
            w = IP_OK | L4_CHECKED
        elif k % 4 == 2 and fam == 4:
            p[rng.choice([1, 4, 5, 8, 10, 11])] ^= 0x40
            w &= ~IP_OK
        pkts.append(bytes(p) + rng.randbytes(rng.choice([0, 3, 17])))
        want.append(w)
    arena, lens, tile_off = _device_batch(pkts)
    ok = engine.rx_verify_device(arena, lens, tile_off).cpu().numpy()
    assert _rx_kernel_waves() == tile_waves
    assert list(ok) == want
    assert (np.array(want) == VERIFIED).sum() > 1000
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_rx_verify_device_edges(oracle, tile_waves):
    """Frames the GPU parser must treat as the host parser does: empty, short,
    malformed and non-IP frames; IPv6 extension headers inside and past the
    80-byte register window; fragments and routing headers (unchecked); UDP
    over IPv4 without a checksum; a truncated TCP header; long link padding; and
    ICMPv4 without a pseudo-header -- an all-zero message with a zero field
    fails (its checksum is 0xFFFF), while a message whose first 8 bytes are zero
    but whose payload sums to 0xFFFF verifies.  Every verdict equals the host
    path's (pipck_rx_verify on the same bytes)."""
    from pip_amd import engine

    rng = random.Random(5)
    zero_icmp = _ipv4(oracle, 1, bytes(8))                        # T = 0: checksum should be 0xFFFF
    ffff_icmp = _ipv4(oracle, 1, bytes(8) + b"\xff\xff")          # T = 0xFFFF: checksum 0, verifies
    cases = [
        (b"", 0), (bytes(19), 0), (bytes([0x45]) + bytes(30), 0), (bytes([0x55]) + bytes(60), 0),
        (_rx_packet(oracle, rng, 6, 6, 200, 1, ext=_ext([(0, 0), (60, 1)], 6)), VERIFIED),
        (_rx_packet(oracle, rng, 6, 17, 300, 2, ext=_ext([(0, 20), (60, 3)], 17)), VERIFIED),  # past 80 B
        (_rx_packet(oracle, rng, 6, 58, 64, 3, ext=_ext([(44, 0)], 58)), VERIFIED),   # atomic fragment
        (_rx_packet(oracle, rng, 6, 17, 200, 4, ext=_ext([(44, 0x0001)], 17)), UNCHECKED),
        (_rx_packet(oracle, rng, 6, 6, 200, 5, ext=_ext([(43, 0)], 6)), UNCHECKED),   # routing header
        (_rx_packet(oracle, rng, 4, 6, 40, 6, frag=0x2000), UNCHECKED),
        (_rx_packet(oracle, rng, 4, 17, 100, 7), UNCHECKED),                          # k % 7 == 0: no UDP sum
        (_rx_packet(oracle, rng, 4, 1, 8, 8), VERIFIED),
        (_rx_packet(oracle, rng, 4, 6, 40, 9)[:20 + 12], None),                       # truncated TCP
        (_rx_packet(oracle, rng, 4, 6, 20, 10) + bytes(100), VERIFIED),               # long link padding
        (_rx_packet(oracle, rng, 6, 6, 20, 11) + rng.randbytes(90), VERIFIED),
        (zero_icmp, IP_OK | L4_CHECKED), (ffff_icmp, VERIFIED),
    ]
    frames = [p for p, _ in cases]
    lib, q = _rxq()
    try:
        bufs = [C.create_string_buffer(p, max(len(p), 1)) for p in frames]
        host = _run(lib, q, [C.cast(b, C.c_void_p).value for b in bufs], [len(p) for p in frames])
    finally:
        lib.pipck_rxq_destroy(q)
    arena, lens, tile_off = _device_batch(frames)
    dev = engine.rx_verify_device(arena, lens, tile_off).cpu().numpy()
    assert list(dev) == list(host)
    for (p, w), got in zip(cases, dev):
        if w is not None:
            assert got == w, (p[:48].hex(), got, w)
    # a tile holding a frame under 16 bytes reads its headers from memory; the
    # others take them from the stream (k_packedb_rx's capture): both, here
    keep = [i for i, p in enumerate(frames) if len(p) >= 16]
    arena, lens, tile_off = _device_batch([frames[i] for i in keep])
    dev2 = engine.rx_verify_device(arena, lens, tile_off).cpu().numpy()
    assert _rx_kernel_waves() == tile_waves
    assert list(dev2) == [host[i] for i in keep]


@pytest.mark.gpu
def test_rx_verify_device_bounded_by_the_arena(oracle, tile_waves):
    """A tile index that claims more bytes than the arena holds: that tile is
    not read, its packets get 0 and PIPCK_ERANGE is set (no Python guard: the
    C ABI directly)."""
    import torch

    from pip_amd import _lib

    rng = random.Random(9)
    frames = [_rx_packet(oracle, rng, 4, 6, 500, k + 1) for k in range(130)]
    arena, lens, tile_off = _device_batch(frames)
    n = len(frames)
    ok = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    short = int(tile_off[1].item()) + 10  # tile 0 fits, tiles 1 and 2 do not
    lib = _lib.load()
    rc = lib.pipck_rx_verify_device(arena.data_ptr(), short, lens.data_ptr(), tile_off.data_ptr(), n,
                                    ok.data_ptr(), err.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    got = ok.cpu().numpy()
    assert (got[:64] == VERIFIED).all() and (got[64:] == 0).all()
    assert int(err.item()) & (1 << _lib.PIPCK_ERANGE)


@pytest.mark.gpu
def test_rx_verify_device_full_size(tile_waves):
    """BASELINE scale (8M frames, cfg4's Zipf lengths, 8.5 GB): frames whose
    TCP/UDP and IPv4 header checksums this engine's ragged kernel filled in
    (engine.gen_rx_frames) all verify -- except UDP/IPv4 frames whose checksum
    came out 0x0000, sent as "no checksum" and reported unchecked -- and one
    flipped byte in 4,000 sampled frames fails exactly the checksum covering
    it (a checksum-of-checksum property: two kernels, sizes the oracle cannot
    reach)."""
    import torch

    from pip_amd import engine

    n = 8 << 20
    arena, lens, tile_off, kind, start, l4 = engine.gen_rx_frames(n, 77)
    hl = torch.where(kind == 3, 40, 20)
    field = start + hl + torch.where(kind == 2, 6, 16)
    no_sum = (kind == 2) & (arena[field] == 0) & (arena[field + 1] == 0)
    want = torch.full((n,), VERIFIED, dtype=torch.uint8, device="cuda")
    want[no_sum] = UNCHECKED
    ok = engine.rx_verify_device(arena, lens, tile_off)
    assert _rx_kernel_waves() == tile_waves
    assert torch.equal(ok, want), int((ok != want).sum().item())
    # one byte flipped: an L4 payload byte (not the checksum field) or an IPv4 TTL
    g = torch.Generator(device="cuda").manual_seed(5)
    pick = torch.randperm(n, device="cuda", generator=g)[:4000]
    pick = pick[~no_sum[pick]]
    half = pick.numel() // 2
    l4_pick, ip_pick = pick[:half], pick[half:]
    ip_pick = ip_pick[kind[ip_pick] != 3]
    where = start[l4_pick] + hl[l4_pick] + 18 + (torch.rand(half, device="cuda", generator=g) *
                                                (l4[l4_pick] - 18).to(torch.float32)).to(torch.int64)
    arena[where] ^= 0x10
    arena[start[ip_pick] + 8] ^= 0x01
    want[l4_pick] = IP_OK | L4_CHECKED
    want[ip_pick] = VERIFIED & ~IP_OK
    ok = engine.rx_verify_device(arena, lens, tile_off)
    assert torch.equal(ok, want), int((ok != want).sum().item())


@pytest.mark.gpu
def test_host_rx_verify_packed_equals_rx_verify(oracle):
    """pipck_host_rx_verify_packed (frames back to back in host memory, DMA'd
    in chunks and judged by pipck_rx_verify_device) gives pipck_rx_verify's
    bits: the 5,000-packet batch with damage and padding (several 64-MiB
    chunks when repeated), from pinned and from pageable memory, plus the edge
    frames (empty, short: the lane-per-segment tiles)."""
    from pip_amd import _lib

    rng = random.Random(404)
    frames, want = [], []
    for k in range(5000):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        l4len = rng.randint(8000, 9000) if k % 20 == 0 else rng.randint(20, 1500)
        p = bytearray(_rx_packet(oracle, rng, fam, proto, l4len, k + 1))
        checked = not (fam == 4 and proto == 17 and (k + 1) % 7 == 0)
        w = VERIFIED if checked else UNCHECKED
        hl = 20 if fam == 4 else 40
        if k % 3 == 1 and checked:
            i = rng.randrange(hl + 18, len(p)) if len(p) > hl + 18 else hl
            p[i] ^= 0x20
            w = IP_OK | L4_CHECKED
        frames.append(bytes(p) + rng.randbytes(rng.choice([0, 5])))
        want.append(w)
    frames = frames * 15  # ~110 MB: more than one 64-MiB chunk
    want = want * 15
    frames += [b"", bytes(10), _rx_packet(oracle, rng, 4, 1, 8, 9)]
    want += [0, 0, VERIFIED]
    lib = _lib.load()
    blob = b"".join(frames)
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    ctx = C.c_void_p()
    assert lib.pipck_ctx_create(-1, C.byref(ctx)) == 0
    try:
        for pinned in (True, False):
            if pinned:
                p = lib.pipck_host_alloc(len(blob))
                C.memmove(p, blob, len(blob))
                base = p
            else:
                buf = np.frombuffer(blob, dtype=np.uint8).copy()
                base = buf.ctypes.data
            ok = np.full(len(frames), 0xEE, dtype=np.uint8)
            good = C.c_uint64(99)
            rc = lib.pipck_host_rx_verify_packed(ctx, base, lens.ctypes.data, len(frames), ok.ctypes.data,
                                                 C.byref(good))
            assert rc == 0, lib.pipck_last_error()
            assert list(ok) == want, pinned
            assert good.value == int((ok == VERIFIED).sum())
            if pinned:
                assert lib.pipck_host_free(C.c_void_p(p)) == 0
    finally:
        lib.pipck_ctx_destroy(ctx)


@pytest.mark.gpu
def test_rx_device_parser_fuzz_equals_host_parser(oracle):
    """Differential fuzz of the two parsers (the host's rx_parse + k_rx_verify,
    and the GPU's rx_from_window): 20,000 frames mutated from valid packets --
    random IHL / total length / payload length / fragment field / protocol /
    next-header chains, truncation, padding, bytes flipped anywhere -- must get
    identical bits from pipck_rx_verify (scattered, host-parsed) and from
    pipck_rx_verify_device (byte-packed in HBM, parsed on the GPU), both with
    and without tiles of short frames."""
    from pip_amd import engine

    rng = random.Random(77)
    frames = []
    for k in range(20000):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1, 58, 47]) if fam == 4 else rng.choice([6, 17, 58, 1, 50])
        ext = b""
        if fam == 6 and rng.random() < 0.3:
            chain = [(rng.choice([0, 60, 44, 43]), rng.choice([0, 1, 3, 20])) for _ in range(rng.randint(1, 3))]
            chain = [(t, a if t != 44 else rng.choice([0, 1, 8])) for t, a in chain]
            ext = _ext(chain, proto)
        p = bytearray(_rx_packet(oracle, rng, fam, proto, rng.randint(0, 300), k + 1, ext=ext,
                                 frag=rng.choice([0, 0, 0, 0x2000, 0x0010]) if fam == 4 else 0))
        for _ in range(rng.choice([0, 0, 1, 2])):  # mutate header fields or any byte
            i = rng.randrange(0, min(len(p), 64)) if rng.random() < 0.7 else rng.randrange(len(p))
            p[i] = rng.randrange(256)
        r = rng.random()
        if r < 0.1:
            p = p[:rng.randrange(0, len(p) + 1)]  # truncated
        elif r < 0.2:
            p += rng.randbytes(rng.randint(1, 120))  # link padding
        frames.append(bytes(p))
    lib, q = _rxq()
    try:
        bufs = [C.create_string_buffer(f, max(len(f), 1)) for f in frames]
        host = _run(lib, q, [C.cast(b, C.c_void_p).value for b in bufs], [len(f) for f in frames])
    finally:
        lib.pipck_rxq_destroy(q)
    arena, lens, tile_off = _device_batch(frames)
    dev = engine.rx_verify_device(arena, lens, tile_off).cpu().numpy()
    bad = np.nonzero(dev != host)[0]
    assert bad.size == 0, [(int(i), frames[i][:64].hex(), int(host[i]), int(dev[i])) for i in bad[:3]]
    keep = [i for i, f in enumerate(frames) if len(f) >= 16]  # every tile streamed (header windows captured)
    arena, lens, tile_off = _device_batch([frames[i] for i in keep])
    dev2 = engine.rx_verify_device(arena, lens, tile_off).cpu().numpy()
    bad = np.nonzero(dev2 != host[keep])[0]
    assert bad.size == 0, [(int(keep[i]), frames[keep[i]][:64].hex(), int(host[keep[i]]), int(dev2[i])) for i in bad[:3]]
    assert len(set(host.tolist())) >= 6  # the fuzz reaches many verdicts


def _ring(frames, stride):
    import torch

    buf = np.zeros(len(frames) * stride, dtype=np.uint8)
    for i, f in enumerate(frames):
        buf[i * stride:i * stride + len(f)] = np.frombuffer(f, dtype=np.uint8)
    lens = torch.from_numpy(np.array([len(f) for f in frames], dtype=np.uint16).view(np.int16)).to("cuda")
    return torch.from_numpy(buf).to("cuda"), lens


# pipck_rx_verify_ring's three schedules (pipck_rxdev.hip): the default slot
# groups (k_ring), the row stream (k_ring_rx, tune flag bit 28) and slot by slot
# (k_ring_slots, the wave-per-packet arm)
RING_KERNELS = {"groups": "k_ring<8, 12>", "own": "k_ring<8, 12>", "coop": "k_ring<8, 12>", "rows": "k_ring_rx",
                "slots": "k_ring_slots"}


def _ring_schedule(name):
    from pip_amd import engine

    if name == "rows":
        engine.tune(alt_flat_schedule=True)
    elif name == "slots":
        engine.tune(lanes_per_packet=256)
    elif name == "own":  # k_ring's row stream: each wave its own 16 slots
        engine.tune(ring_own_slots=True, ring_adapt=False)
    elif name == "coop":  # k_ring's row stream: items dealt round-robin to the block's waves
        engine.tune(ring_all_coop=True, ring_adapt=False)
    else:  # "groups": k_ring itself, whatever the ring's earlier launches reported
        engine.tune(ring_adapt=False)


def _ring_frames(oracle, rng, stride, fill, count):
    """count oracle-checksummed IPv4/IPv6 TCP/UDP/ICMP frames that fit the slot,
    every third damaged, some with link padding.  fill "mixed": L4 lengths up to
    the slot; "dense": within ~200 B of filling the slot (k_ring's interleaved row stream),
    with a run of short frames every 512; "short": frames in runs of 16 whose longest is <= 128 / 256 / 512
    bytes or up to the slot, so k_ring's waves take every schedule (S = 8, 16, 32
    lanes per slot, and the row stream)."""
    frames = []
    for k in range(count):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        hl = 20 if fam == 4 else 40
        cap = stride if fill != "short" else (128, 256, 512, stride)[(k // 16) % 4]
        top = min(9000, cap - hl - 7)
        lo = max(20, top - 200) if fill == "dense" and (k // 64) % 8 != 5 else 20
        l4len = rng.randint(lo, top)
        p = bytearray(_rx_packet(oracle, rng, fam, proto, l4len, k + 1))
        if k % 3 == 1:
            p[rng.randrange(len(p))] ^= 0x04
        frames.append(bytes(p) + rng.randbytes(rng.choice([0, 0, 7])))
    return frames


def _host_bits(frames):
    lib, q = _rxq()
    try:
        bufs = [C.create_string_buffer(f, max(len(f), 1)) for f in frames]
        return _run(lib, q, [C.cast(b, C.c_void_p).value for b in bufs], [len(f) for f in frames])
    finally:
        lib.pipck_rxq_destroy(q)


@pytest.mark.gpu
@pytest.mark.parametrize("fill", ["mixed", "short", "dense"])
@pytest.mark.parametrize("schedule", ["groups", "own", "coop", "rows", "slots"])
@pytest.mark.parametrize("stride", [1024, 2048, 9216])
def test_rx_verify_ring_equals_host_path(oracle, stride, schedule, fill):
    """pipck_rx_verify_ring (frames in fixed-size slots of a device ring, the unused
    rest of each slot never read) gives pipck_rx_verify's bits under each of its
    schedules: oracle-checksummed IPv4/IPv6 TCP/UDP/ICMP frames with damage and
    link padding, edge frames (empty, short, malformed, extension headers past
    the register window)."""
    from pip_amd import engine

    rng = random.Random(stride * 3 + len(fill))
    frames = _ring_frames(oracle, rng, stride, fill, 3000)
    frames += [b"", bytes(10), bytes([0x45]) + bytes(30), _rx_packet(oracle, rng, 4, 1, 8, 9),
               _rx_packet(oracle, rng, 6, 17, 300, 2, ext=_ext([(0, 20), (60, 3)], 17))]
    host = _host_bits(frames)
    ring, lens = _ring(frames, stride)
    _ring_schedule(schedule)
    try:
        dev = engine.rx_verify_ring(ring, stride, lens).cpu().numpy()
        assert RING_KERNELS[schedule] in _last_kernel()
    finally:
        engine.tune()
    bad = np.nonzero(dev != host)[0]
    assert bad.size == 0, [(int(i), frames[i][:48].hex(), int(host[i]), int(dev[i])) for i in bad[:3]]
    assert (host == VERIFIED).sum() > 1000


def _last_kernel():
    buf = C.create_string_buffer(4096)
    from pip_amd import _lib

    _lib.check("pipck_last_launch", _lib.load().pipck_last_launch(buf, len(buf)))
    return buf.value.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("schedule", ["groups", "rows", "slots"])
def test_rx_verify_ring_full_size(schedule):
    """2M Zipf frames (engine.gen_rx_frames, checksummed by the ragged kernel) in
    9,216-byte slots: every frame verifies but the zero-checksum UDP ones, and the
    ring's verdicts equal the byte-packed path's on the same frames."""
    import torch

    from pip_amd import engine

    n, stride = 2 << 20, 9216
    ring, lens, kind = engine.gen_rx_ring(n, 31, stride)
    _ring_schedule(schedule)
    try:
        ok = engine.rx_verify_ring(ring, stride, lens)
        assert RING_KERNELS[schedule] in _last_kernel()
    finally:
        engine.tune()
    arena, lens2, tile_off, _, _, _ = engine.gen_rx_frames(n, 31)
    ok2 = engine.rx_verify_device(arena, lens2, tile_off)
    assert torch.equal(ok, ok2)
    n_ok = int((ok == VERIFIED).sum().item())
    assert n_ok > n - 100 and int((ok == UNCHECKED).sum().item()) == n - n_ok


@pytest.mark.gpu
@pytest.mark.parametrize("stride,l4_len", [(1024, 100), (2048, 200), (1536, 1480), (9216, 8900)])
def test_rx_verify_ring_dense_and_short_full_size(stride, l4_len):
    """The bench rings (tools/rx_device_bench.py) at 1M slots: short frames in small
    slots and full slots, under all three schedules -- identical verdicts, every
    frame verified but zero-checksum UDP."""
    import torch

    from pip_amd import engine

    n = 1 << 20
    ring, lens, kind = engine.gen_rx_ring(n, 5, stride, l4_len=l4_len)
    got = {}
    for schedule in RING_KERNELS:
        _ring_schedule(schedule)
        try:
            got[schedule] = engine.rx_verify_ring(ring, stride, lens).clone()
            assert RING_KERNELS[schedule] in _last_kernel()
        finally:
            engine.tune()
    assert all(torch.equal(got["groups"], got[k]) for k in got)
    ok = got["groups"]
    n_ok = int((ok == VERIFIED).sum().item())
    assert n_ok > n - 1000 and int((ok == UNCHECKED).sum().item()) == n - n_ok


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [1024, 2048, 4080, 4096, 9216])
def test_rx_verify_ring_default_schedule(oracle, stride):
    """The ring's default schedule is the slot groups (k_ring) at every slot size,
    and its verdicts equal the other two schedules' on the same ring: 1,001
    oracle-checksummed frames, a third damaged, n not a multiple of any wave's
    slots."""
    from pip_amd import engine

    rng = random.Random(stride + 7)
    frames = []
    for k in range(1001):
        fam = rng.choice([4, 6])
        p = bytearray(_rx_packet(oracle, rng, fam, rng.choice([6, 17]), rng.randint(20, stride - 80), k + 1))
        if k % 3 == 1:
            p[rng.randrange(len(p))] ^= 0x10
        frames.append(bytes(p))
    ring, lens = _ring(frames, stride)
    dev = engine.rx_verify_ring(ring, stride, lens).cpu().numpy()
    # the first launch on a ring is k_ring; from 4 KiB slots a later one may take
    # the row stream when this address's earlier launches (another test's ring
    # at a reused address) reported full slots
    assert RING_KERNELS["groups"] in _last_kernel() or (stride >= 4096 and "k_ring_rx" in _last_kernel())
    for schedule in ("own", "coop", "rows", "slots"):
        _ring_schedule(schedule)
        try:
            other = engine.rx_verify_ring(ring, stride, lens).cpu().numpy()
            assert RING_KERNELS[schedule] in _last_kernel()
        finally:
            engine.tune()
        assert np.array_equal(dev, other), schedule
    assert 600 < int((dev == VERIFIED).sum()) < 700


@pytest.mark.gpu
@pytest.mark.parametrize("stride", [4096, 9216])
def test_rx_verify_ring_adapts_to_the_fill(stride):
    """The default schedule of jumbo-slot rings follows the ring's own fill: a ring
    of full slots starts on k_ring and, once a launch has reported its fill (a
    synchronise in between), takes the row stream k_ring_rx; when the same ring
    (same address) then holds short frames, it goes back to k_ring.  Every launch
    gives the verdicts k_ring gives (tune ring_adapt=False) on the same bytes."""
    import torch

    from pip_amd import engine

    n = 64 * 1000 + 37
    engine.tune()
    try:
        ring, lens, _ = engine.gen_rx_ring(n, 17, stride, l4_len=stride - 300)
        engine.tune(ring_adapt=False)
        want = engine.rx_verify_ring(ring, stride, lens).clone()
        assert "k_ring<8, 12>" in _last_kernel()
        engine.tune()
        kernels = []
        for _ in range(6):
            got = engine.rx_verify_ring(ring, stride, lens)
            kernels.append(_last_kernel())
            torch.cuda.synchronize()
            assert torch.equal(got, want)
        assert "k_ring_rx" in kernels[-1], kernels
        # the same ring now holds short frames only: back to k_ring
        short = torch.minimum(lens.to(torch.int32) & 0xFFFF, torch.tensor(300, device=lens.device)).to(torch.int16)
        engine.tune(ring_adapt=False)
        want2 = engine.rx_verify_ring(ring, stride, short).clone()
        engine.tune()
        kernels = []
        for _ in range(6):
            got = engine.rx_verify_ring(ring, stride, short)
            kernels.append(_last_kernel())
            torch.cuda.synchronize()
            assert torch.equal(got, want2)
        assert "k_ring<8, 12>" in kernels[-1], kernels
        # a sparse ring (Zipf frames in 9 KiB slots, 220-B frames in 4 KiB) stays on
        # k_ring once it has reported (its first launch may follow an earlier
        # test's dense ring freed at the same address), verdicts unchanged
        ring3, lens3, _ = engine.gen_rx_ring(n, 19, stride, l4_len=0 if stride >= 9216 else 200)
        engine.tune(ring_adapt=False)
        want3 = engine.rx_verify_ring(ring3, stride, lens3).clone()
        engine.tune()
        kernels = []
        for _ in range(4):
            got = engine.rx_verify_ring(ring3, stride, lens3)
            kernels.append(_last_kernel())
            torch.cuda.synchronize()
            assert torch.equal(got, want3)
        assert all("k_ring<8, 12>" in k for k in kernels[1:]), kernels
    finally:
        engine.tune()


@pytest.mark.gpu
def test_rx_verify_ring_feedback_recycles_entries():
    """More jumbo-slot rings than the feedback remembers (64): the least recently
    used entries are recycled, and every call still gives k_ring's verdicts --
    full rings and sparse ones interleaved at distinct addresses."""
    import torch

    from pip_amd import engine

    stride, n = 4096, 64 * 3 + 5
    rings = []
    for k in range(70):
        ring, lens, _ = engine.gen_rx_ring(n, 100 + k, stride, l4_len=stride - 300 if k % 2 else 200)
        engine.tune(ring_adapt=False)
        want = engine.rx_verify_ring(ring, stride, lens).clone()
        engine.tune()
        rings.append((ring, lens, want))
    try:
        for _ in range(3):
            for ring, lens, want in rings:
                got = engine.rx_verify_ring(ring, stride, lens)
                torch.cuda.synchronize()
                assert torch.equal(got, want)
    finally:
        engine.tune()
