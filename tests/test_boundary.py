"""GPU: link-substitution boundary test.

oracle/_ref/stack_replay_amd is pip's REAL TCP/UDP/IP stack (compiled from
/root/reference without pip_checksum.cpp) linked against the product's
libpip_checksum_amd.so.  It replays a scripted exchange -- IPv4 and IPv6 TCP
handshakes (SYN-ACK with its 8-byte option segment), multi-segment writes,
odd-length data, UDP over v4/v6 with odd and jumbo payloads, all-zero and
all-0xFF datagrams -- and prints every IP packet pip emits.  The bytes must
equal what pip emits with its own pip_checksum.cpp (tests/golden/stack_replay.txt,
recorded from oracle/_ref/stack_replay_ref).
"""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REPLAY_AMD = ROOT / "oracle" / "_ref" / "stack_replay_amd"
GOLDEN = ROOT / "tests" / "golden" / "stack_replay.txt"


def test_golden_replay_is_self_consistent():
    lines = GOLDEN.read_text().strip().splitlines()
    assert lines[-1] == f"PACKETS {len(lines) - 1} VERIFY_BAD 0"
    assert len(lines) - 1 >= 25


def _without_ip_id(line: str) -> str:
    """A hex IPv4 packet line with ip_id and ip_sum replaced by the header's
    validity (its RFC 1071 sum folds to 0xFFFF); other lines unchanged."""
    try:
        p = bytearray.fromhex(line)
    except ValueError:
        return line
    if len(p) < 20 or p[0] >> 4 != 4:
        return line
    ihl = (p[0] & 15) * 4
    s = sum(p[i] << 8 | p[i + 1] for i in range(0, ihl, 2))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    p[4] = p[5] = p[10] = 0
    p[11] = int(s == 0xFFFF)
    return p.hex()


@pytest.mark.gpu
@pytest.mark.parametrize("capture", [False, True])
def test_pip_stack_on_amd_checksum_is_byte_identical(capture):
    """capture: the same replay with the drop-in's capture mode on -- pip's
    unchanged call sites queue their checksums and one flush per stack action
    fills them before the packets are emitted."""
    import os

    assert REPLAY_AMD.exists(), "build with `make -C oracle ref ref-amd` where /root/reference exists"
    env = dict(os.environ)
    if capture:
        env["PIPCK_REPLAY_CAPTURE"] = "1"
    r = subprocess.run([str(REPLAY_AMD)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    want = GOLDEN.read_text().strip().splitlines()
    got = r.stdout.strip().splitlines()
    resends = [int(ln.split()[1]) for ln in r.stderr.splitlines() if ln.startswith("RESENDS")]
    assert resends, r.stderr[-2000:]
    if resends[0]:  # pip's timer race shifted the ip_ids: compare without them (stack_replay.cpp)
        got, want = [_without_ip_id(ln) for ln in got], [_without_ip_id(ln) for ln in want]
    extra = [ln[:120] for ln in got if ln not in want]
    assert got[-1] == want[-1], (extra, [ln[:120] for ln in want if ln not in got])
    diff = [i for i, (a, b) in enumerate(zip(got, want)) if a != b]
    assert not diff and len(got) == len(want), diff[:5]
    # the deferred (batched) API on real pip_buf chains, flushed in one GPU batch
    # and pipelined: submitted every 5 packets while the next are queued, then completed
    lines = [ln for ln in r.stderr.splitlines() if ln.startswith("DEFERRED")]
    # and zero-copy from pinned memory with every chain reference dropped before the flush
    assert [ln.split()[2] for ln in lines] == ["flush", "pipelined", "zero_copy"], r.stderr[-2000:]
    for line in lines:
        f = line.split()
        assert f[f.index("bad") + 1] == "0" and f[f.index("pending_after") + 1] == "0", line
        assert int(f[f.index("checked") + 1]) >= 25
    zc = lines[-1].split()
    assert zc[zc.index("free_while_queued") + 1] == "6"  # PIPCK_EBUSY
    assert zc[zc.index("free_after") + 1] == "0"


@pytest.mark.gpu
@pytest.mark.parametrize("family,mss", [(4, 1460), (4, 8960), (6, 1440)])
def test_pip_tx_path_at_volume_matches_pip(family, mss):
    """pip's TCP write() path at volume over IPv4 and IPv6 (oracle/stack_tx_bench.cpp): pip's own
    build vs the drop-in synchronously, in capture mode, with zero-copy, and
    pipelined across two connections -- FNV-1a over every emitted wire byte must
    be identical (the IPv4 ip_id aside when pip's own timer race drew one, see
    same()), and pip's 1-s retransmission must never fire."""
    import json
    import os

    ref_bin = ROOT / "oracle" / "_ref" / "stack_tx_ref"
    amd_bin = ROOT / "oracle" / "_ref" / "stack_tx_amd"
    assert ref_bin.exists() and amd_bin.exists(), "build with `make -C oracle ref ref-amd`"

    def run(binary, *args):
        cmd = [str(binary), "--family", str(family), "--mss", str(mss), "--bytes", str(8 << 20), "--write", str(1 << 20),
               "--verify", *args]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=dict(os.environ))
        # exit 3 = pip's timer resent a segment that had waited >= 1 s for its ACK: a stall
        assert r.returncode == 0, (args, r.stderr[-2000:])
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["retransmits"] == 0 and d["digest_of"] == "every wire byte"
        # no segment came near pip's 1 s resend (pip_tcp_check.cpp:30); resends of younger
        # segments are pip's own timer race (stale_clock_resends, also in pip's build:
        # profiles/r04_pip_timer_race.jsonl) and never reach the digested wire bytes
        assert d["max_unacked_ms"] < 500 and d["max_action_ms"] < 500, d
        print(binary.name, args, {k: d[k] for k in ("max_action_ms", "max_action", "max_unacked_ms",
                                                    "stale_clock_resends", "cold_ms")})
        return d

    def same(a, b, what):
        # every wire byte except the IPv4 ip_id / ip_sum fields, and every IPv4
        # header's validity -- always; every byte -- when pip's timer fired in
        # neither run: a stale-clock resend draws an ip_id from pip_netif's
        # shared counter (pip/pip_netif.cpp:90) and shifts every later packet's
        # ip_id and ip_sum, in pip's own build as in the drop-in's
        assert (a["digest_noid"], a["packets"]) == (b["digest_noid"], b["packets"]), what
        if a["stale_clock_resends"] == 0 and b["stale_clock_resends"] == 0:
            assert a["digest"] == b["digest"], what

    for conns in ("1", "2"):
        want = run(ref_bin, "--conns", conns)
        modes = [("--mode", "capture"), ("--mode", "capture_zc")]
        if conns == "1":
            modes.append(("--mode", "sync"))
        else:
            modes.append(("--mode", "capture_zc", "--pipeline"))
        for m in modes:
            same(run(amd_bin, "--conns", conns, *m), want, (conns, m))


def test_tx_bench_on_pips_own_build_reports_resend_ages():
    """CPU: pip's own build (no drop-in, no GPU) through the same TX driver --
    the JSON line carries the stall metrics the drop-in runs are judged by, and
    a resend by pip's timer is only ever classed as a stall when the segment
    had waited >= 1 s (pip_tcp_check.cpp:25-39; the race at :45-56 resends
    younger ones, profiles/r04_pip_timer_race.jsonl)."""
    import json

    ref_bin = ROOT / "oracle" / "_ref" / "stack_tx_ref"
    if not ref_bin.exists():
        pytest.skip("oracle/_ref is built where /root/reference exists")
    for family in (4, 6):
        r = subprocess.run([str(ref_bin), "--family", str(family), "--mss", "1460", "--bytes", str(64 << 20),
                            "--write", str(1 << 20), "--conns", "2"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["retransmits"] == 0 and d["max_unacked_ms"] < 500 and d["max_action"] in (
            "write", "ack input", "syn -> syn-ack", "handshake ack", "flush")
        assert d["stale_clock_resends"] >= 0 and (d["stale_clock_resends"] == 0) == (d["max_resend_age_ms"] == 0)
        assert d["packets"] > (64 << 20) // 1460
    # the ip_id-independent digest (stack_tx_bench.cpp digest_noid) of two runs of
    # pip's own build agrees even when pip's timer raced in one of them
    runs = []
    for _ in range(2):
        r = subprocess.run([str(ref_bin), "--family", "4", "--mss", "1460", "--bytes", str(16 << 20), "--write",
                            str(1 << 20), "--conns", "2", "--verify"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert runs[0]["digest_noid"] == runs[1]["digest_noid"] and runs[0]["packets"] == runs[1]["packets"]
    if runs[0]["stale_clock_resends"] == runs[1]["stale_clock_resends"] == 0:
        assert runs[0]["digest"] == runs[1]["digest"]


def test_ip_id_normalisation_keeps_header_validity():
    """_without_ip_id (the stack replay's comparison under pip's timer race):
    ip_id and ip_sum give way to the header's validity, everything else stays."""
    import struct

    def v4(ident, good):
        h = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 28, ident, 0x4000, 64, 17, 0, b"\x0a\0\0\x01",
                                  b"\x0a\0\0\x02"))
        s = sum(h[i] << 8 | h[i + 1] for i in range(0, 20, 2))
        while s >> 16:
            s = (s & 0xFFFF) + (s >> 16)
        h[10:12] = struct.pack(">H", (~s & 0xFFFF) ^ (0 if good else 1))
        return (bytes(h) + b"\x01\x02\x03\x04\x05\x06\x07\x08").hex()

    assert _without_ip_id(v4(1, True)) == _without_ip_id(v4(2, True))
    assert _without_ip_id(v4(1, True)) != _without_ip_id(v4(1, False))
    six = "60000000000811400000000000000000000000000000000100000000000000000000000000000002" + "00" * 8
    assert _without_ip_id(six) == six and _without_ip_id("PACKETS 3") == "PACKETS 3"


@pytest.mark.gpu
@pytest.mark.parametrize("family,length", [(6, 8952), (4, 8972), (4, 1472)])
def test_pip_udp_tx_path_matches_pip(family, length):
    """pip's UDP send path (pip_udp::output, pip/protocol/pip_udp.cpp:28-64) at
    volume through oracle/stack_udp_bench.cpp: pip's own build vs the drop-in
    synchronously, in capture mode, with zero-copy and pipelined batches --
    FNV-1a over every emitted wire byte must be identical."""
    import json

    ref_bin = ROOT / "oracle" / "_ref" / "stack_udp_ref"
    amd_bin = ROOT / "oracle" / "_ref" / "stack_udp_amd"
    assert ref_bin.exists() and amd_bin.exists(), "build with `make -C oracle ref ref-amd`"

    def run(binary, nbytes, *args):
        r = subprocess.run([str(binary), "--family", str(family), "--len", str(length), "--bytes", str(nbytes),
                            "--verify", *args], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, (args, r.stderr[-2000:])
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert d["digest_of"] == "every wire byte" and d["datagrams"] == nbytes // length
        return d["digest"]

    assert run(amd_bin, 4 << 20, "--mode", "sync") == run(ref_bin, 4 << 20)
    want = run(ref_bin, 16 << 20)
    for args in (("--mode", "capture"), ("--mode", "capture_zc"), ("--mode", "capture_zc", "--pipeline"),
                 ("--mode", "capture_zc", "--pipeline", "--batch", "1000")):
        assert run(amd_bin, 16 << 20, *args) == want, args


def _verify(packets):
    """pip_checksum_amd_verify_packets (the drop-in's RX batch verifier) over Python bytes,
    once with every packet in its own buffer and once with the packets back to back in
    one buffer (the drop-in then takes the chunked-DMA path): the same bits both ways."""
    import ctypes as C

    import numpy as np

    from pip_amd import _lib

    lib = C.CDLL(str(_lib.LIBSHIM))
    fn = lib.pip_checksum_amd_verify_packets
    fn.restype = C.c_uint32
    fn.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_void_p]
    lens = (C.c_uint32 * len(packets))(*[len(p) for p in packets])
    bufs = [C.create_string_buffer(bytes(p), max(len(p), 1)) for p in packets]
    ptrs = (C.c_void_p * len(packets))(*[C.cast(b, C.c_void_p) for b in bufs])
    ok = np.zeros(len(packets), dtype=np.uint8)
    good = fn(ptrs, lens, len(packets), ok.ctypes.data)
    assert good == int((ok == VERIFIED).sum())
    blob = C.create_string_buffer(b"".join(bytes(p) for p in packets), max(sum(len(p) for p in packets), 1))
    base, offs = C.cast(blob, C.c_void_p).value, np.cumsum([0] + [len(p) for p in packets[:-1]])
    ptrs2 = (C.c_void_p * len(packets))(*[base + int(o) for o in offs])
    ok2 = np.zeros(len(packets), dtype=np.uint8)
    good2 = fn(ptrs2, lens, len(packets), ok2.ctypes.data)
    assert good2 == good and np.array_equal(ok2, ok), np.nonzero(ok2 != ok)[0][:5]
    return ok


# ok bits of pip_checksum_amd_verify_packets (include/pip_checksum_amd.h)
IP_OK, L4_OK, L4_CHECKED = 1, 2, 4
VERIFIED, UNCHECKED = 7, 3


@pytest.mark.gpu
def test_rx_verify_accepts_what_pip_emits_and_rejects_corruption():
    """SURVEY 8 f2 on pip's own packets: every IPv4/IPv6 TCP/UDP packet pip's
    real stack emits (tests/golden/stack_replay.txt, pip's build) verifies in
    one GPU batch; flipping any one byte of a packet's IPv4 header or TCP/UDP
    segment is caught in the right bit; truncated or non-IP packets get 0."""
    import random

    import numpy as np

    pkts = [bytes.fromhex(l.strip()) for l in GOLDEN.read_text().splitlines() if l.strip() and
            not l.startswith(("PACKETS", "VERIFY"))]
    assert len(pkts) >= 20
    assert (_verify(pkts) == VERIFIED).all()
    rng = random.Random(7)
    bad, where = [], []
    for p in pkts:
        v4 = p[0] >> 4 == 4
        hl = (p[0] & 15) * 4 if v4 else 40
        # a byte of the IPv4 header that only its own checksum covers (TOS, id, TTL, the
        # checksum itself; not the fragment field, which would make it a fragment whose
        # payload is left unchecked), or a byte of the TCP/UDP segment
        i = rng.choice([1, 4, 5, 8, 10, 11] if v4 and rng.random() < 0.5 else list(range(hl, len(p))))
        q = bytearray(p)
        q[i] ^= 0x10
        bad.append(bytes(q))
        where.append(1 if i < hl else 2)
    ok = _verify(bad)
    for o, w in zip(ok, where):
        assert o == VERIFIED - w, (o, w)  # exactly the damaged checksum fails; the payload was still checked
    junk = [b"", bytes(10), bytes([0x45]) + bytes(10), bytes([0x45, 0, 0xFF, 0xFF]) + bytes(16), bytes([0x60]) + bytes(20)]
    assert (_verify(junk) == 0).all()
    # a thread whose FIRST drop-in call is the verifier, then exits: its RX queue is
    # torn down before its HIP context (thread_local destruction order)
    import threading

    res = {}
    t = threading.Thread(target=lambda: res.setdefault("ok", _verify(pkts)))
    t.start()
    t.join()
    assert (res["ok"] == VERIFIED).all()


def _rx_packet(oracle, rng, fam, proto, l4len, k, good=True, ext=b"", frag=0):
    """An IPv4/IPv6 packet whose checksums the oracle (pip's arithmetic) filled in:
    TCP/UDP over their pseudo-headers, ICMPv4 over the message alone
    (pip_ip_checksum), ICMPv6 over the IPv6 pseudo-header (next header 58).
    ext: IPv6 extension headers before the upper layer, as _ext() returns them;
    frag: IPv4 ip_off."""
    import struct

    l4 = bytearray(rng.randbytes(l4len))
    src, dst = rng.randbytes(4 if fam == 4 else 16), rng.randbytes(4 if fam == 4 else 16)
    field = {6: 16, 17: 6, 1: 2, 58: 2}.get(proto)
    if field is not None and l4len >= field + 2:
        l4[field:field + 2] = b"\0\0"
        if fam == 4 and proto == 17 and k % 7 == 0:
            pass  # no UDP checksum over IPv4 (RFC 768): the field stays 0
        else:
            if proto == 1:
                c = oracle.ip_checksum(bytes(l4))
            elif fam == 4:
                c = oracle.inet_checksum(bytes(l4), proto, src, dst, l4len)
            else:
                c = oracle.inet6_checksum(bytes(l4), proto, src, dst, l4len)
            if fam == 4 and proto == 17 and c == 0:
                c = 0xFFFF  # never "no checksum" by accident (either verifies: both mean zero)
            l4[field:field + 2] = struct.pack(">H", c)
    if fam == 4:
        hdr = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, 20 + l4len, k & 0xFFFF, frag or 0x4000, 64, proto, 0,
                                    src, dst))
        hdr[10:12] = struct.pack(">H", oracle.ip_checksum(bytes(hdr)))
    else:
        chain, first = ext if ext else (b"", proto)
        hdr = bytearray(struct.pack(">IHBB16s16s", 0x60000000, len(chain) + l4len, first, 64, src, dst))
        ext = chain
    return bytes(hdr) + bytes(ext) + bytes(l4)


def _ext(chain, upper):
    """IPv6 extension headers: chain = [(type, arg)] in order -- arg is the
    fragment field (offset << 3 | M) for a fragment header (44), else the
    Hdr Ext Len (the header is 8 * (arg + 1) bytes, PadN-filled); returns the
    bytes and the first header's type (the fixed header's next header)."""
    import struct

    out = b""
    types = [t for t, _ in chain] + [upper]
    for i, (t, arg) in enumerate(chain):
        nxt = types[i + 1]
        if t == 44:  # fragment header: next, reserved, offset<<3 | M, identification
            out += struct.pack(">BBHI", nxt, 0, arg, 0x1234)
        else:  # hop-by-hop / destination options / routing: (len+1)*8 bytes, PadN filled
            n = 8 * (arg + 1)
            out += bytes([nxt, arg]) + bytes([1, n - 4]) + bytes(n - 4)
    return out, types[0]


@pytest.mark.gpu
def test_rx_verify_against_the_oracle(oracle):
    """Random TCP/UDP over IPv4 and IPv6 packets whose checksums the oracle
    (pip's arithmetic) filled in -- odd lengths, options, UDP over IPv4 without
    a checksum, ICMP -- all verify; the same packets with a wrong L4 checksum
    fail bit 1 only."""
    import random
    import struct

    import numpy as np

    rng = random.Random(11)
    good, checked = [], []
    for k in range(3000):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        l4len = rng.randint(20 if proto == 6 else 8, 3000)
        p = _rx_packet(oracle, rng, fam, proto, l4len, k)
        good.append(p + rng.randbytes(rng.choice([0, 0, 6])))  # trailing link padding
        checked.append(not (fam == 4 and proto == 17 and k % 7 == 0))
    ok = _verify(good)
    for o, c in zip(ok, checked):
        assert o == (VERIFIED if c else UNCHECKED), o
    broken = []
    for p in good:
        v4 = p[0] >> 4 == 4
        hl = 20 if v4 else 40
        proto = p[9] if v4 else p[6]
        field = {6: 16, 17: 6, 1: 2, 58: 2}[proto]
        q = bytearray(p)
        if not (v4 and proto == 17 and q[hl + 6] == 0 and q[hl + 7] == 0):
            q[hl + field] ^= 0x01
        broken.append(bytes(q))
    ok = _verify(broken)
    for c, o in zip(checked, ok):
        # a damaged TCP / UDP / ICMPv4 / ICMPv6 checksum: checked, and only its bit fails
        assert o == (IP_OK | L4_CHECKED if c else UNCHECKED), o


@pytest.mark.gpu
def test_rx_verify_fragments_extension_headers_and_other_protocols(oracle):
    """What the verifier cannot check from one packet is reported as unchecked
    (ok == 3, PIP_RX_L4_CHECKED clear), never as verified: IPv4 fragments (MF or
    an offset; their L4 checksum spans the reassembled datagram), IPv6 fragment
    and routing headers, protocols without a known checksum.  IPv6 hop-by-hop /
    destination-options headers and atomic fragments are walked to the upper
    layer and checked."""
    import random

    rng = random.Random(5)
    cases = []
    for k in range(40):
        proto = [6, 17, 1][k % 3]
        # IPv4 fragments carrying garbage where an L4 header would be: header checked only
        for frag in (0x2000, 0x0010, 0x2010, 0x1FFF):
            p = bytearray(_rx_packet(oracle, rng, 4, proto, 64, k + 1, frag=frag))
            p[30:34] = b"\xde\xad\xbe\xef"  # any L4 bytes: not checkable here (the header's checksum still holds)
            cases.append((bytes(p), UNCHECKED))
        p6 = [6, 17, 58][k % 3]
        # walked to the upper layer and checked
        for chain in ([(0, 0)], [(60, 1)], [(0, 0), (60, 0)], [(44, 0)], [(0, 1), (44, 0)]):
            cases.append((_rx_packet(oracle, rng, 6, p6, 100 + k, k, ext=_ext(chain, p6)), VERIFIED))
        # not checkable from one packet
        for chain in ([(44, 0x0001)], [(44, 0x00A8)], [(43, 0)], [(0, 0), (43, 1)]):
            cases.append((_rx_packet(oracle, rng, 6, p6, 100 + k, k, ext=_ext(chain, p6)), UNCHECKED))
        # protocols without a checksum this knows (GRE, ESP; IPv6 next header 1 is not ICMPv6)
        cases.append((_rx_packet(oracle, rng, 4, 47, 40, k), UNCHECKED))
        cases.append((_rx_packet(oracle, rng, 6, 50, 40, k), UNCHECKED))
        cases.append((_rx_packet(oracle, rng, 6, 1, 40, k), UNCHECKED))
    ok = _verify([c for c, _ in cases])
    for (p, want), o in zip(cases, ok):
        assert o == want, (p[:48].hex(), o, want)
    # the walked ones really are checked: damage the upper layer's checksum field
    walked = [p for p, w in cases if w == VERIFIED]
    bad = []
    for p in walked:
        q = bytearray(p)
        nh, at = q[6], 40
        while nh in (0, 60, 44):
            nh, at = q[at], at + (8 if nh == 44 else 8 * (q[at + 1] + 1))
        q[at + {6: 16, 17: 6, 58: 2}[nh]] ^= 0x40
        bad.append(bytes(q))
    assert (_verify(bad) == IP_OK | L4_CHECKED).all()
    # an extension header whose length runs past the payload: malformed, no L4 bits
    p = bytearray(_rx_packet(oracle, rng, 6, 6, 40, 1, ext=_ext([(0, 0)], 6)))
    p[41] = 30  # hop-by-hop Hdr Ext Len: 248 bytes, past the 48-byte payload
    assert list(_verify([bytes(p)])) == [IP_OK]
    # truncated ICMP (under 8 bytes) and TCP headers: no L4 bits
    short = [_rx_packet(oracle, rng, 4, 1, 4, 1), _rx_packet(oracle, rng, 6, 58, 6, 1), _rx_packet(oracle, rng, 4, 6, 12, 1)]
    assert list(_verify(short)) == [IP_OK, IP_OK, IP_OK]


@pytest.mark.gpu
def test_rx_verify_reads_pinned_packets_in_place(oracle):
    """Packets that lie in pinned memory (a tun read ring from pipck_host_alloc)
    are read in place by the RX queue (auto zero-copy): same verdicts as the
    same packets on the heap, at odd alignments inside the ring, mixed with heap
    packets in one call, and after the ring is freed nothing refers to it."""
    import ctypes as C
    import random

    import numpy as np

    from pip_amd import _lib

    rng = random.Random(23)
    pkts = []
    for k in range(600):
        fam = rng.choice([4, 6])
        proto = rng.choice([6, 17, 1]) if fam == 4 else rng.choice([6, 17, 58])
        p = bytearray(_rx_packet(oracle, rng, fam, proto, rng.randint(20, 1500), k + 1))
        if k % 5 == 0:
            p[-1] ^= 0x20  # damaged payload byte: its L4 checksum fails
        pkts.append(bytes(p))
    heap_ok = _verify(pkts)
    lib = _lib.load()
    size = sum(len(p) + 7 for p in pkts) + 64
    base = lib.pipck_host_alloc(size)
    assert base
    try:
        ptrs, off = [], 3  # odd start: packets at arbitrary alignments
        for i, p in enumerate(pkts):
            C.memmove(base + off, p, len(p))
            ptrs.append(base + off)
            off += len(p) + (i % 7)
        fn = C.CDLL(str(_lib.LIBSHIM)).pip_checksum_amd_verify_packets
        fn.restype = C.c_uint32
        fn.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_uint32), C.c_uint32, C.c_void_p]
        heap = [C.create_string_buffer(p, len(p)) for p in pkts]
        # every other packet from the pinned ring, the rest from the heap
        mix = [C.c_void_p(ptrs[i]) if i % 2 == 0 else C.cast(heap[i], C.c_void_p) for i in range(len(pkts))]
        arr = (C.c_void_p * len(pkts))(*mix)
        lens = (C.c_uint32 * len(pkts))(*[len(p) for p in pkts])
        ok = np.zeros(len(pkts), dtype=np.uint8)
        good = fn(arr, lens, len(pkts), ok.ctypes.data)
        assert np.array_equal(ok, heap_ok) and good == int((ok == VERIFIED).sum())
        assert (ok == VERIFIED).sum() > 300 and (ok == IP_OK | L4_CHECKED).sum() >= 100  # damaged: checked, failed
    finally:
        assert lib.pipck_host_free(base) == 0  # nothing still holds the ring
