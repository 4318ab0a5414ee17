"""GPU: the packed-batch C ABI bounds every tile by the arena on the device
(pipck_{checksum,verify}_packed{,_bytes}_n, include/pipck.h) -- VERDICT r03 item 5.

The calls go straight through ctypes, with no Python-side guard: an index that
places a tile (64 packets) past the arena -- a stale or foreign tile_off /
tile_chunk, or lengths that no longer match it -- must read nothing there,
report PIPCK_ERANGE in d_err and give 0 for that tile's packets, while every
other tile's results stay those of the untampered batch."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from pip_amd import _lib, engine  # noqa: E402
from pip_amd.workloads import CFG4, N_FLOWS  # noqa: E402

pytestmark = pytest.mark.gpu
ERANGE_BIT = 1 << 2  # 1 << PIPCK_ERANGE


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def _run(fn, arena, arena_bytes, lens, index, n, pseudo, verify):
    lib = _lib.load()
    out = torch.zeros(n, dtype=torch.uint8 if verify else torch.int16, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = getattr(lib, fn)(_p(arena), C.c_uint64(arena_bytes), _p(lens), _p(index), C.c_uint64(n), _p(pseudo),
                          C.c_uint32(N_FLOWS), C.c_void_p(0), C.c_uint64(0), _p(out), _p(err), C.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, _lib.load().pipck_last_error()
    return out.cpu().numpy().view(np.uint8 if verify else np.uint16), int(err.item())


@pytest.mark.parametrize("layout", ["bytes", "packed16"])
@pytest.mark.parametrize("verify", [False, True])
def test_index_past_the_arena_is_an_error_not_a_fault(layout, verify):
    n = 64 * 40 + 17  # 41 tiles, the last one partial
    w = CFG4
    if layout == "bytes":
        arena, lens, index, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_bytes_n" if verify else "pipck_checksum_packed_bytes_n"
        unit = 1
    else:
        arena, lens, index, _ = engine.gen_packed(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_n" if verify else "pipck_checksum_packed_n"
        unit = 16
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    nbytes = arena.numel()
    good, err0 = _run(fn, arena, nbytes, lens, index, n, pseudo, verify)
    assert err0 == 0
    if not verify:  # the bounded call equals the plain (trusted-index) one on a correct index
        plain = (engine.checksum_packed_bytes if layout == "bytes" else engine.checksum_packed)(
            arena, lens, index, n, pseudo, N_FLOWS)
        assert np.array_equal(plain.cpu().numpy().view(np.uint16), good)
    total = int(index[(n + 63) // 64].item())  # bytes (or chunks) of the whole batch
    bad = index.clone()
    bad[5] = total * 1000 + 12345            # far past the arena
    bad[9] = total - 3                        # starts inside, its packets run past the end
    bad[13] = (1 << 62) + 7                   # would overflow an unchecked offset + length
    got, err = _run(fn, arena, nbytes, lens, bad, n, pseudo, verify)
    assert err == ERANGE_BIT
    flagged = np.zeros(n, dtype=bool)
    for t in (5, 9, 13):
        flagged[64 * t:64 * t + 64] = True
    assert (got[flagged] == 0).all()
    assert np.array_equal(got[~flagged], good[~flagged])
    # an arena shorter than the index claims: the tail tiles are refused the same way
    short = (total * unit) // 2
    got, err = _run(fn, arena, short, lens, index, n, pseudo, verify)
    assert err == ERANGE_BIT
    limit = short if unit == 1 else (short + 15) // 16  # the arena's bytes, or its 16-byte chunks
    tiles_ok = [t for t in range((n + 63) // 64) if int(index[t + 1].item()) <= limit]
    assert 0 < len(tiles_ok) < (n + 63) // 64
    for t in range((n + 63) // 64):
        sl = slice(64 * t, min(n, 64 * t + 64))
        if t in tiles_ok:
            assert np.array_equal(got[sl], good[sl]), t
        else:
            assert (got[sl] == 0).all(), t
    # lengths grown after the index was built: the last tile now reaches past the end
    lens2 = lens.clone()
    lens2[n - 1] = -1  # 65535 as u16
    got, err = _run(fn, arena, nbytes, lens2, index, n, pseudo, verify)
    assert err == ERANGE_BIT and (got[64 * 40:] == 0).all()
    assert np.array_equal(got[:64 * 40], good[:64 * 40])


# ---------------------------------------------------------------------------
# the ring, ragged and chain ABIs bound their indices too
# ---------------------------------------------------------------------------
def _hip():
    return C.CDLL("libamdhip64.so")


class _ExactBuffer:
    """Device memory from hipMalloc of exactly `size` bytes (no caching-allocator
    slack after it), filled from host bytes."""

    def __init__(self, data: bytes):
        self.hip = _hip()
        self.ptr = C.c_void_p()
        assert self.hip.hipMalloc(C.byref(self.ptr), C.c_size_t(len(data))) == 0
        assert self.hip.hipMemcpy(self.ptr, C.c_char_p(data), C.c_size_t(len(data)), 1) == 0  # H2D

    def free(self):
        self.hip.hipFree(self.ptr)


def _ipv4_frame(oracle, rng, l4len, k, total_override=None):
    from tests.test_boundary import _rx_packet

    p = bytearray(_rx_packet(oracle, rng, 4, 6, l4len, k))
    if total_override is not None:
        p[2], p[3] = total_override >> 8, total_override & 0xFF
    return bytes(p)


@pytest.mark.parametrize("schedule", ["groups", "own", "coop", "rows", "slots"])
@pytest.mark.parametrize("stride", [1024, 9216])
def test_ring_length_past_the_slot_is_an_error_not_a_fault(oracle, schedule, stride):
    """pipck_rx_verify_ring_n through ctypes, no Python guard, on a ring hipMalloc'd
    as exactly n * stride bytes: the LAST slot claims 65,535 B and carries an IPv4
    total length past the slot; a middle slot claims stride + 16 B over a frame that
    would verify; another claims exactly the stride (allowed).  The two refused slots
    get verdict 0 and d_err = 1 << PIPCK_ERANGE; every other slot equals the host
    path (pipck_rx_verify) on the same bytes, under each of the ring's schedules."""
    import random

    from tests.test_gpu_rx import RING_KERNELS, _host_bits, _last_kernel, _ring_frames, _ring_schedule

    rng = random.Random(stride + 99)
    n = 256 + 77  # several waves / blocks of every schedule, the last one partial
    frames = _ring_frames(oracle, rng, stride, "short" if stride == 1024 else "mixed", n)
    full = _ipv4_frame(oracle, rng, stride - 20, 5)  # exactly one slot
    frames[100] = full
    frames[n - 1] = _ipv4_frame(oracle, rng, 400, 7, total_override=stride + 500)  # IP total past the slot
    frames[n - 2] = _ipv4_frame(oracle, rng, 300, 8)
    host = _host_bits(frames)
    blob = bytearray(n * stride)
    for i, f in enumerate(frames):
        blob[i * stride:i * stride + len(f)] = f
    lens = np.array([len(f) for f in frames], dtype=np.uint16)
    lens[n - 1] = 65535          # the last slot: far past the slot (and the ring)
    lens[40] = stride + 16       # a middle slot: into the next slot
    ring = _ExactBuffer(bytes(blob))
    try:
        dl = torch.from_numpy(lens.view(np.int16)).to("cuda")
        ok = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        lib = _lib.load()
        _ring_schedule(schedule)
        try:
            rc = lib.pipck_rx_verify_ring_n(ring.ptr, C.c_uint64(stride), _p(dl), C.c_uint64(n), _p(ok), _p(err),
                                            C.c_void_p(0))
            assert rc == 0, lib.pipck_last_error()
            torch.cuda.synchronize()
            assert RING_KERNELS[schedule] in _last_kernel()
        finally:
            engine.tune()
        got = ok.cpu().numpy()
        assert int(err.item()) == ERANGE_BIT
        assert got[n - 1] == 0 and got[40] == 0
        keep = np.ones(n, dtype=bool)
        keep[[40, n - 1]] = False
        bad = np.nonzero(got[keep] != host[keep])[0]
        assert bad.size == 0, bad[:5]
        assert host[100] == 7 and got[100] == 7  # a frame filling its slot exactly is judged normally
        # the untampered lengths: nothing refused, the middle slot judged again
        lens_ok = np.array([len(f) for f in frames], dtype=np.uint16)
        err.zero_()
        dl_ok = torch.from_numpy(lens_ok.view(np.int16)).to("cuda")  # held across the call
        rc = lib.pipck_rx_verify_ring_n(ring.ptr, C.c_uint64(stride), _p(dl_ok), C.c_uint64(n), _p(ok), _p(err),
                                        C.c_void_p(0))
        assert rc == 0
        torch.cuda.synchronize()
        assert int(err.item()) == 0 and np.array_equal(ok.cpu().numpy(), host)
    finally:
        ring.free()


def _ragged_case(n_flows=8):
    rng = np.random.default_rng(123)
    size = 300_000
    host = rng.integers(0, 256, size, dtype=np.uint8)
    arena = torch.from_numpy(host).to("cuda")
    n = 64 * 5 + 9
    offs = rng.integers(0, size - 9000, n).astype(np.uint64)
    lens = rng.integers(0, 9000, n).astype(np.uint32)
    flows = rng.integers(0, n_flows, n).astype(np.uint32)
    return host, arena, offs, lens, flows


def _tamper(offs, lens, flows, size, n_flows):
    offs, lens, flows = offs.copy(), lens.copy(), flows.copy()
    bad = {3: "far", 70: "straddles", 71: "overflow", 150: "flow", 200: "ends_exactly", 328: "len0_past"}
    offs[3] = size * 100
    offs[70], lens[70] = size - 10, 20
    offs[71], lens[71] = (1 << 64) - 8, 64
    flows[150] = n_flows + 3
    offs[200], lens[200] = size - 64, 64  # ends exactly at the arena's end: allowed
    offs[328], lens[328] = size + 1, 0     # empty, but past the end (the last descriptor)
    refused = [i for i, why in bad.items() if why != "ends_exactly"]
    return offs, lens, flows, refused


@pytest.mark.parametrize("arm", ["default", "wave"])
@pytest.mark.parametrize("verify", [False, True])
def test_ragged_descriptor_past_the_arena_is_an_error_not_a_fault(oracle, verify, arm):
    """pipck_{checksum,verify}_ragged_n through ctypes: descriptors far past the
    arena, straddling its end, overflowing offset + len, naming a flow past the
    table, or empty past the end are not read -- result 0 (verify 0), d_err =
    1 << PIPCK_ERANGE -- while every other descriptor's result equals the
    untampered call's, under the default kernel and the wave-per-packet arm."""
    n_flows = 8
    host, arena, offs, lens, flows = _ragged_case(n_flows)
    size = host.size
    _, pseudo = engine.gen_flows(4, n_flows, 77, 6)
    lib = _lib.load()
    fn = "pipck_verify_ragged_n" if verify else "pipck_checksum_ragged_n"

    def run(o, ln, fl):
        desc = engine.make_desc(o, ln, fl)
        out = torch.zeros(len(o), dtype=torch.uint8 if verify else torch.int16, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        rc = getattr(lib, fn)(_p(arena), C.c_uint64(size), _p(desc), C.c_uint64(len(o)), _p(pseudo),
                              C.c_uint32(n_flows), _p(out), _p(err), C.c_void_p(0))
        torch.cuda.synchronize()
        assert rc == 0, lib.pipck_last_error()
        return out.cpu().numpy().view(np.uint8 if verify else np.uint16), int(err.item())

    if arm == "wave":
        engine.tune(lanes_per_packet=256)
    try:
        good, err0 = run(offs, lens, flows)
        assert err0 == 0
        o2, l2, f2, refused = _tamper(offs, lens, flows, size, n_flows)
        # the reference results of the tampered-but-legal descriptor (200)
        ref, _ = run(o2[[200]], l2[[200]], f2[[200]])
        got, err = run(o2, l2, f2)
    finally:
        engine.tune()
    assert err == ERANGE_BIT
    assert (got[refused] == 0).all()
    same = np.setdiff1d(np.arange(len(offs)), refused + [200])
    assert np.array_equal(got[same], good[same])
    assert got[200] == ref[0]
    if not verify:  # the oracle agrees on a sample (pip_inet_checksum with the flow's pseudo-header)
        seg = host[int(o2[200]):int(o2[200]) + int(l2[200])].tobytes()
        s, d = oracle.flow4(77, int(f2[200]))
        assert got[200] == oracle.inet_checksum(seg, 6, s, d)


def test_chains_bounded_by_arena_segments_and_flows(oracle):
    """pipck_checksum_chains_n through ctypes: a packet holding one segment past the
    arena, a packet whose segment range runs past n_segs, one whose range is
    reversed, and one whose flow is past the table get 0 and set d_err; every
    other packet equals the oracle's pip_inet_checksum_buf."""
    rng = np.random.default_rng(5)
    n_pk, n_flows, seed, proto = 300, 8, 4242, 6
    seg_lens, seg_begin = [], [0]
    for _ in range(n_pk):
        seg_lens += [int(rng.integers(0, 1500)) for _ in range(int(rng.integers(1, 5)))]
        seg_begin.append(len(seg_lens))
    seg_lens = np.array(seg_lens, dtype=np.uint32)
    offs = np.zeros(len(seg_lens), dtype=np.uint64)
    pos = 0
    for i, L in enumerate(seg_lens):
        offs[i] = pos
        pos += int(L) + int(rng.integers(0, 9))
    host = rng.integers(0, 256, pos, dtype=np.uint8)
    arena = torch.from_numpy(host).to("cuda")
    _, pseudo = engine.gen_flows(4, n_flows, seed, proto)
    pkt_flow = rng.integers(0, n_flows, n_pk).astype(np.int32)
    # tamper: packet 10's second segment past the arena, packet 50's flow, packets
    # 120 (range past n_segs) and 121 (reversed range) -- the last packet ranges kept legal
    n_segs = len(seg_lens)
    offs[seg_begin[10] + 1 if seg_begin[11] - seg_begin[10] > 1 else seg_begin[10]] = pos + 5000
    pkt_flow[50] = n_flows
    sb = np.array(seg_begin, dtype=np.int64)
    sb_bad = sb.copy()
    sb_bad[121] = n_segs + 40  # packet 120: [sb[120], n_segs + 40) passes n_segs; packet 121: reversed
    refused = [10, 50, 120, 121]
    segs = engine.make_desc(offs, seg_lens, np.zeros(n_segs))
    scratch = torch.empty(n_segs, dtype=torch.int32, device="cuda")
    out = torch.zeros(n_pk, dtype=torch.int16, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    lib = _lib.load()
    d_sb, d_flow = torch.from_numpy(sb_bad).to("cuda"), torch.from_numpy(pkt_flow).to("cuda")  # held across the call
    rc = lib.pipck_checksum_chains_n(_p(arena), C.c_uint64(host.size), _p(segs), C.c_uint64(n_segs), _p(d_sb),
                                     _p(d_flow), C.c_uint64(n_pk), _p(pseudo), C.c_uint32(n_flows), _p(scratch),
                                     _p(out), _p(err), C.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, lib.pipck_last_error()
    got = out.cpu().numpy().view(np.uint16)
    assert int(err.item()) == ERANGE_BIT
    assert (got[refused] == 0).all()
    for p in range(n_pk):
        if p in refused:
            continue
        chain = [host[int(offs[s]):int(offs[s]) + int(seg_lens[s])].tobytes() for s in range(sb[p], sb[p + 1])]
        s, d = oracle.flow4(seed, int(pkt_flow[p]))
        assert got[p] == oracle.inet_checksum_chain(chain, proto, s, d), p


@pytest.mark.parametrize("layout", ["bytes", "packed16"])
@pytest.mark.parametrize("verify", [False, True])
def test_flow_of_entry_past_the_table_is_an_error(layout, verify):
    """pipck_*_packed{,_bytes}_n with a per-packet flow table (d_flow_of) and
    n_flows > 0: an entry >= n_flows (a stale or foreign flow index) gives its
    packet 0 and sets PIPCK_ERANGE -- pseudo[] is never read there -- while
    every other packet equals the run with valid entries."""
    n = 64 * 12 + 5
    w = CFG4
    if layout == "bytes":
        arena, lens, index, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_bytes_n" if verify else "pipck_checksum_packed_bytes_n"
    else:
        arena, lens, index, _ = engine.gen_packed(n, 0, w.seed, w.hdr)
        fn = "pipck_verify_packed_n" if verify else "pipck_checksum_packed_n"
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    rng = np.random.default_rng(3)
    flows = rng.integers(0, N_FLOWS, n).astype(np.int32)
    lib = _lib.load()

    def run(fl):
        d_fl = torch.from_numpy(fl).to("cuda")  # held across the call
        out = torch.zeros(n, dtype=torch.uint8 if verify else torch.int16, device="cuda")
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        rc = getattr(lib, fn)(_p(arena), C.c_uint64(arena.numel()), _p(lens), _p(index), C.c_uint64(n), _p(pseudo),
                              C.c_uint32(N_FLOWS), _p(d_fl), C.c_uint64(0), _p(out), _p(err), C.c_void_p(0))
        torch.cuda.synchronize()
        assert rc == 0, lib.pipck_last_error()
        return out.cpu().numpy().view(np.uint8 if verify else np.uint16), int(err.item())

    good, err0 = run(flows)
    assert err0 == 0
    bad_at = [0, 63, 64, 400, n - 1]
    fl2 = flows.copy()
    fl2[bad_at] = [N_FLOWS, 1 << 30, N_FLOWS + 1, -1, 5000]  # -1: 0xFFFFFFFF as u32
    got, err = run(fl2)
    assert err == ERANGE_BIT
    assert (got[bad_at] == 0).all()
    keep = np.setdiff1d(np.arange(n), bad_at)
    assert np.array_equal(got[keep], good[keep])


# ---------------------------------------------------------------------------
# the fixed-stride flow index is bounded on the device too
# ---------------------------------------------------------------------------
# (stride, len, arena offset, tune, kernel): every fixed launch shape that reads
# a flow_of entry, each asserted by name through pipck_last_launch
FIXED_SHAPES = {
    "coop_cfg2": (1488, 1480, 0, {}, "k_flat_coop<32"),
    "coop_jumbo": (8992, 8980, 0, {}, "k_flat_coop<32"),
    "flat_1k": (1024, 1000, 0, {}, "k_flat<24"),
    "flat_alt": (1488, 1480, 0, {"alt_flat_schedule": True}, "k_flat<24"),
    "flat_small": (256, 250, 0, {}, "k_flat_small<16"),
    "flat_tiny": (40, 36, 0, {}, "k_flat_tiny<4"),
    "small": (44, 40, 0, {}, "k_small<"),
    "fixed": (1001, 999, 3, {}, "k_fixed<"),
    "wave": (1488, 1480, 0, {"lanes_per_packet": 256}, "k_wave<"),
}


def _fixed_call(fn, arena, stride, length, n, pseudo, n_flows, flow_of, verify):
    lib = _lib.load()
    out = torch.full((n,), 0x5A, dtype=torch.uint8 if verify else torch.int16, device="cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    args = [_p(arena), C.c_uint64(stride), C.c_uint32(length), C.c_uint64(n), _p(pseudo), C.c_uint32(n_flows),
            _p(flow_of), C.c_uint64(0), _p(out)]
    rc = getattr(lib, fn)(*args, *([_p(err)] if fn.endswith("_n") else []), C.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0, lib.pipck_last_error()
    from tests.test_gpu_rx import _last_kernel

    return out.cpu().numpy().view(np.uint8 if verify else np.uint16), int(err.item()), _last_kernel()


@pytest.mark.parametrize("shape", list(FIXED_SHAPES))
@pytest.mark.parametrize("verify", [False, True])
def test_fixed_flow_of_entry_past_the_table_is_an_error(oracle, shape, verify):
    """pipck_{checksum,verify}_fixed_n through ctypes, no Python guard: flow_of
    entries >= n_flows planted at a block task's first and last packet and at the
    batch's last packet (plus 0xFFFFFFFF and 2^30) give their packets 0 (verify 0)
    and d_err = 1 << PIPCK_ERANGE, the pseudo table is never read there, and every
    other packet equals the run with valid entries -- which equals the trusted
    plain call and pip's pip_inet_checksum (oracle) -- under every fixed launch
    shape, the kernel asserted by name."""
    stride, length, off, knobs, kname = FIXED_SHAPES[shape]
    n, n_flows, seed, proto = 64 * 13 + 29, 8, 901, 6
    rng = np.random.default_rng(len(shape) * 7 + stride)
    host = rng.integers(0, 256, off + n * stride + 64, dtype=np.uint8)
    base = torch.from_numpy(host).to("cuda")
    arena = base[off:]
    _, pseudo = engine.gen_flows(4, n_flows, seed, proto)
    flows = rng.integers(0, n_flows, n).astype(np.int32)
    fn = "pipck_verify_fixed" if verify else "pipck_checksum_fixed"
    engine.tune(**knobs)
    try:
        d_fl = torch.from_numpy(flows).to("cuda")
        good, err0, k0 = _fixed_call(fn + "_n", arena, stride, length, n, pseudo, n_flows, d_fl, verify)
        plain, _, _ = _fixed_call(fn, arena, stride, length, n, pseudo, n_flows, d_fl, verify)
        # block tasks of 128 packets (k_flat_coop at 1,488 B), 24 (jumbo), wave tasks of 16-64:
        # every such boundary below is a first or last packet of some task
        bad_at = sorted({0, 23, 24, 63, 64, 127, 128, 255, 256, 383, 384, n - 2, n - 1})
        fl2 = flows.copy()
        fl2[bad_at] = [n_flows, 1 << 30, -1, n_flows + 1] * 3 + [n_flows]  # -1: 0xFFFFFFFF as u32
        d_fl2 = torch.from_numpy(fl2).to("cuda")
        got, err, k1 = _fixed_call(fn + "_n", arena, stride, length, n, pseudo, n_flows, d_fl2, verify)
    finally:
        engine.tune()
    assert kname in k0 and kname in k1, (k0, k1)
    assert err0 == 0 and np.array_equal(good, plain)
    assert err == ERANGE_BIT
    assert (got[bad_at] == 0).all()
    keep = np.setdiff1d(np.arange(n), bad_at)
    assert np.array_equal(got[keep], good[keep])
    if verify:
        return
    for i in list(range(0, n, 97)) + [n - 3]:
        pkt = host[off + i * stride:off + i * stride + length].tobytes()
        s, d = oracle.flow4(seed, int(flows[i]))
        assert good[i] == oracle.inet_checksum(pkt, proto, s, d), i


def test_fixed_n_requires_n_flows():
    """The bounded fixed forms refuse n_flows == 0 with a pseudo table (the plain
    form with flow_of ignores n_flows, as before)."""
    lib = _lib.load()
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    _, pseudo = engine.gen_flows(4, 4, 1, 6)
    fl = torch.zeros(2, dtype=torch.int32, device="cuda")
    out = torch.zeros(2, dtype=torch.int16, device="cuda")
    rc = lib.pipck_checksum_fixed_n(_p(arena), C.c_uint64(1488), C.c_uint32(1480), C.c_uint64(2), _p(pseudo),
                                    C.c_uint32(0), _p(fl), C.c_uint64(0), _p(out), C.c_void_p(0), C.c_void_p(0))
    assert rc == _lib.PIPCK_EINVAL
    rc = lib.pipck_checksum_fixed(_p(arena), C.c_uint64(1488), C.c_uint32(1480), C.c_uint64(2), _p(pseudo),
                                  C.c_uint32(0), _p(fl), C.c_uint64(0), _p(out), C.c_void_p(0))
    torch.cuda.synchronize()
    assert rc == 0


def test_engine_flow_of_defaults_to_the_whole_table(oracle):
    """an engine call with flow_of and no n_flows bounds the entries by
    the whole pseudo table (pseudo.numel()), never by 1 -- fixed, packed and
    byte-packed forms give every packet its flow's checksum."""
    n, n_flows, seed, proto, stride, length = 300, 16, 77, 6, 1488, 1480
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, n * stride, dtype=np.uint8)
    arena = torch.from_numpy(host).to("cuda")
    _, pseudo = engine.gen_flows(4, n_flows, seed, proto)
    flows = rng.integers(0, n_flows, n).astype(np.int32)
    d_fl = torch.from_numpy(flows).to("cuda")
    err = torch.zeros(1, dtype=torch.int32, device="cuda")
    got = engine.checksum_fixed(arena, stride, length, n, pseudo, flow_of=d_fl, err=err).cpu().numpy().view(np.uint16)
    for i in range(0, n, 13):
        s, d = oracle.flow4(seed, int(flows[i]))
        assert got[i] == oracle.inet_checksum(host[i * stride:i * stride + length].tobytes(), proto, s, d), i
    w = CFG4
    pa, lens, index, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
    a = engine.checksum_packed_bytes(pa, lens, index, n, pseudo, flow_of=d_fl, err=err)
    b = engine.checksum_packed_bytes(pa, lens, index, n, pseudo, n_flows, flow_of=d_fl, err=err)
    pa16, lens16, index16, _ = engine.gen_packed(n, 0, w.seed, w.hdr)
    c = engine.checksum_packed(pa16, lens16, index16, n, pseudo, flow_of=d_fl, err=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(a, b) and torch.equal(a, c)
    assert int((a != 0).sum().item()) > n - 5


def _update_case(n, stride, length, seed, proto, n_flows, rng):
    host = rng.integers(0, 256, n * stride, dtype=np.uint8)
    host.reshape(n, stride)[:, 16:18] = 0  # th_sum is zero while pip sums the segment
    arena = torch.from_numpy(host).to("cuda")
    _, p_old = engine.gen_flows(4, n_flows, seed, proto)
    _, p_new = engine.gen_flows(4, n_flows, seed ^ 0x5EED, proto)
    flows = rng.integers(0, n_flows, n).astype(np.int32)
    d_fl = torch.from_numpy(flows).to("cuda")
    out = engine.checksum_fixed(arena, stride, length, n, p_old, n_flows, d_fl)
    rows = arena.view(n, stride)
    v = out.to(torch.int32) & 0xFFFF
    rows[:, 16] = (v >> 8).to(torch.uint8)  # th_sum, htons() as pip's callers store it
    rows[:, 17] = (v & 0xFF).to(torch.uint8)
    return arena, p_old, p_new, flows


def test_update_fixed_flow_of_entry_past_the_table_leaves_the_packet(oracle):
    """pipck_update_fixed_n through ctypes: a packet whose flow_of entry is past the
    tables keeps every byte (its edit is not applied, its field not patched) and
    d_err = 1 << PIPCK_ERANGE; every other packet equals the untampered update,
    which equals pip's full recomputation with the new addresses."""
    n, stride, length, seed, proto, n_flows = 64 * 9 + 5, 1488, 1480, 515, 6, 8
    rng = np.random.default_rng(21)
    arena, p_old, p_new, flows = _update_case(n, stride, length, seed, proto, n_flows, rng)
    before = arena.cpu().numpy().copy()
    new = torch.from_numpy(rng.integers(0, 256, n * 8, dtype=np.uint8)).to("cuda")
    lib = _lib.load()

    def run(a, fl):
        err = torch.zeros(1, dtype=torch.int32, device="cuda")
        d_fl = torch.from_numpy(fl).to("cuda")
        rc = lib.pipck_update_fixed_n(_p(a), C.c_uint64(stride), C.c_uint64(n), C.c_uint32(0), C.c_uint32(length),
                                      C.c_uint32(16), C.c_uint32(0), C.c_uint32(8), _p(new), C.c_uint64(8),
                                      _p(p_old), _p(p_new), C.c_uint32(n_flows), _p(d_fl), C.c_uint64(0), _p(err),
                                      C.c_void_p(0))
        torch.cuda.synchronize()
        assert rc == 0, lib.pipck_last_error()
        return a.cpu().numpy(), int(err.item())

    good, err0 = run(arena.clone(), flows)
    assert err0 == 0
    bad_at = [0, 63, 64, 255, n - 1]
    fl2 = flows.copy()
    fl2[bad_at] = [n_flows, -1, -(1 << 31), n_flows + 7, 100]  # -(1 << 31): 0x80000000 as u32
    got, err = run(arena.clone(), fl2)
    assert err == ERANGE_BIT
    g2, b2, h2 = got.reshape(n, stride), good.reshape(n, stride), before.reshape(n, stride)
    assert np.array_equal(g2[bad_at], h2[bad_at])  # refused packets: untouched, every byte
    keep = np.setdiff1d(np.arange(n), bad_at)
    assert np.array_equal(g2[keep], b2[keep])
    # the untampered update equals pip's recomputation over the new bytes and addresses
    for i in list(range(0, n, 41)) + [n - 2]:
        pkt = bytearray(b2[i, :length].tobytes())
        field = (pkt[16] << 8) | pkt[17]
        pkt[16] = pkt[17] = 0
        s, d = oracle.flow4(seed ^ 0x5EED, int(flows[i]))
        assert field == oracle.inet_checksum(bytes(pkt), proto, s, d), i
