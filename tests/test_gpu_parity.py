"""GPU parity: the HIP kernels vs pip (golden fixtures) and vs the oracle.

Everything here runs through libpipck.so on a real MI355X.  Bit-exact is the
bar (integer work).  Sizes: the oracle comparisons use batches the CPU
oracle finishes in seconds; the full BASELINE.json sizes are checked through
size-independent properties (a sampled oracle comparison + checksum-of-checksum:
writing each result into its packet's checksum field must make the packet sum
to 0xFFFF, i.e. recompute to 0x0000 and verify as valid).
"""
import ctypes as C
import hashlib
import json
import threading
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from pip_amd import _lib, engine  # noqa: E402
from pip_amd import checksum as pc  # noqa: E402
from pip_amd.workloads import ALL, CFG1, CFG2, CFG3, CFG4, CFG5, N_FLOWS  # noqa: E402
from tests.golden.make_golden import patch_bytes, run_case  # noqa: E402

DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    engine.require_gpu()
    yield
    engine.tune()
    torch.cuda.synchronize()


def u16(t) -> np.ndarray:
    return t.cpu().numpy().view(np.uint16)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def upload(buf: np.ndarray, misalign: int = 0):
    """Device copy of host bytes starting `misalign` bytes past a 256-B aligned base."""
    t = torch.zeros(buf.size + misalign + 64, dtype=torch.uint8, device=DEV)
    view = t[misalign:misalign + buf.size]
    view.copy_(torch.from_numpy(buf))
    return t, view


class PcAdapter:
    """run_case() adapter: pip's per-packet API on the GPU (pip_amd.checksum)."""

    standard_checksum = staticmethod(lambda d, n, s: pc.pip_standard_checksum(d, n, s))
    ip_checksum = staticmethod(lambda d, n=None: pc.pip_ip_checksum(d, n))
    fold_uint32 = staticmethod(pc.pip_fold_uint32)
    inet_checksum = staticmethod(lambda d, p, s, t, n=None: pc.pip_inet_checksum(d, p, s, t, n))
    inet6_checksum = staticmethod(lambda d, p, s, t, n=None: pc.pip_inet6_checksum(d, p, s, t, n))
    inet_checksum_chain = staticmethod(pc.pip_inet_checksum_buf)
    inet6_checksum_chain = staticmethod(pc.pip_inet6_checksum_buf)


# ----------------------------------------------------------------------------
# 1. pip's known answers through the per-packet (exact) device path
# ----------------------------------------------------------------------------
@pytest.fixture
def staged_per_packet():
    """The per-packet path with staged copies (the default auto mode zero-copies small calls)."""
    pc.set_zero_copy(0)
    yield
    pc.set_zero_copy(2)


def test_every_known_answer_on_gpu(kat, staged_per_packet):
    bad = []
    for c in kat:
        got = run_case(PcAdapter, c)
        if got != c["expect"]:
            bad.append((c["fn"], c.get("data", c.get("segs")), c["expect"], got))
    assert not bad, bad[:5]


def test_every_known_answer_on_gpu_zero_copy(kat):
    """The same known answers through the zero-copy per-packet path (the kernel
    reads pinned host staging and writes the result to host memory)."""
    pc.set_zero_copy(1)
    try:
        bad = [c["fn"] for c in kat if run_case(PcAdapter, c) != c["expect"]]
        assert not bad, bad[:5]
    finally:
        pc.set_zero_copy(2)


@pytest.mark.parametrize("mode", [3, 4])
def test_every_known_answer_on_gpu_resident(kat, mode):
    """The same known answers through the resident service (mode 3: one block
    stays on the GPU polling a doorbell in pinned host memory; mode 4: the
    doorbell in fine-grained device memory; requests over 68 KiB -- the
    131,076-B wrap KATs -- take the staged copies).  The block's idle exit
    and relaunch are exercised too: a pause longer than its 10 ms idle timeout,
    then more calls; then mode changes (each ends the block)."""
    import time

    pc.set_zero_copy(mode)
    try:
        bad = [c["fn"] for c in kat if run_case(PcAdapter, c) != c["expect"]]
        assert not bad, bad[:5]
        time.sleep(0.05)  # the block has exited by now
        small = [c for c in kat if c["fn"] != "fold"][:40]
        bad = [c["fn"] for c in small if run_case(PcAdapter, c) != c["expect"]]
        assert not bad, bad[:5]
        # switching modes ends the block; switching back restarts it
        pc.set_zero_copy(1)
        pc.set_zero_copy(7 - mode)
        pc.set_zero_copy(mode)
        bad = [c["fn"] for c in small if run_case(PcAdapter, c) != c["expect"]]
        assert not bad, bad[:5]
    finally:
        pc.set_zero_copy(2)


def test_per_packet_api_is_thread_safe(kat):
    cases = [c for c in kat if c["fn"] != "fold"][:60]
    errors = []

    def worker():
        try:
            for c in cases:
                if run_case(PcAdapter, c) != c["expect"]:
                    errors.append(c)
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=worker) for _ in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors


# ----------------------------------------------------------------------------
# 2. device generator == fixture bytes; batch kernels == pip's results
# ----------------------------------------------------------------------------
def _device_batch(b, w):
    if w.ragged:
        arena, desc, lens = engine.gen_ragged(b["n"], b["first"], b["seed"], b["hdr"], N_FLOWS)
        return arena, desc, lens
    arena = torch.empty(b["n"] * b["stride"], dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, b["stride"], b["length"], b["n"], b["first"], b["seed"], b["hdr"])
    return arena, None, None


def _pseudo(w, first=0):
    if not w.family:
        return None
    _, pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)
    return pseudo


@pytest.mark.parametrize("name", sorted(ALL))
def test_generator_reproduces_fixture_bytes(batches, name):
    b, w = batches[name], ALL[name]
    arena, desc, lens = _device_batch(b, w)
    torch.cuda.synchronize()
    if w.ragged:
        assert sha(lens.cpu().numpy().astype("<u4")) == b["lengths_sha256"]
        assert arena.numel() == b["arena_bytes"]
    assert sha(arena.cpu().numpy()) == b["arena_sha256"]


def last_kernel() -> str:
    buf = C.create_string_buffer(4096)
    _lib.check("pipck_last_launch", _lib.load().pipck_last_launch(buf, len(buf)))
    return buf.value.decode()


# the kernel each config's bench launch runs: the fixture pins THAT kernel
BENCH_KERNEL = {1: "k_small<", 2: "k_flat_coop<32,", 3: "k_flat_coop<32,", 4: "k_packedb<", 5: "k_flat_coop<32,"}


@pytest.mark.parametrize("name", sorted(ALL))
def test_batch_kernel_reproduces_pips_results(batches, name):
    """pip's own results (compiled pip_checksum.cpp, tests/golden/make_golden.py)
    through the batch kernel and layout the bench runs: cfg1 at the packed 20-B
    stride (k_small at the config's 1M; k_hdr from 8M), cfg4 byte-packed (k_packedb) and 16-B packed (k_packed) and, for the
    descriptor ABI, as ragged descriptors (k_ragged)."""
    b, w = batches[name], ALL[name]
    assert b["stride"] == w.stride
    pseudo = _pseudo(w)
    if w.ragged:
        ab, lb, to, _ = engine.gen_packed_bytes(b["n"], b["first"], b["seed"], b["hdr"])
        assert sha(ab.cpu().numpy()) == b["arena_bytes_sha256"]  # the byte-packed arena pip's results are over
        outs = {"packed_bytes": engine.checksum_packed_bytes(ab, lb, to, b["n"], pseudo, N_FLOWS, None, b["first"])}
        kernel = last_kernel()
        arena, lens16, tc, _ = engine.gen_packed(b["n"], b["first"], b["seed"], b["hdr"])
        outs["packed16"] = engine.checksum_packed(arena, lens16, tc, b["n"], pseudo, N_FLOWS, None, b["first"])
        assert "k_packed<" in last_kernel()
        _, desc, _ = _device_batch(b, w)
        outs["ragged"] = engine.checksum_ragged(arena, desc, pseudo)
        assert "k_ragged<" in last_kernel()
    else:
        arena, _, _ = _device_batch(b, w)
        outs = {"fixed": engine.checksum_fixed(arena, b["stride"], b["length"], b["n"], pseudo, N_FLOWS, None,
                                               b["first"])}
        kernel = last_kernel()
        if w.stride >= 1024:  # the other schedule (k_flat) on the same batch
            engine.tune(alt_flat_schedule=True)
            try:
                outs["k_flat"] = engine.checksum_fixed(arena, b["stride"], b["length"], b["n"], pseudo, N_FLOWS,
                                                       None, b["first"])
                assert "k_flat<" in last_kernel()
            finally:
                engine.tune()
        if w.cfg == 1:  # the header row kernel that batches of >= 8M headers take (k_hdr)
            engine.tune(loads_per_lane=32)
            try:
                outs["hdr"] = engine.checksum_fixed(arena, b["stride"], b["length"], b["n"], pseudo, N_FLOWS, None,
                                                    b["first"])
                assert "k_hdr<5," in last_kernel()
            finally:
                engine.tune()
    assert BENCH_KERNEL[w.cfg] in kernel, kernel
    for path, out in outs.items():
        got = u16(out)
        assert list(got[:16]) == b["head"], path
        assert sha(got.astype("<u2")) == b["results_sha256"], path


EDGES = sorted(k for k in json.loads((Path(__file__).parent / "golden" / "batches.json").read_text())
               if k.startswith("edge_"))


@pytest.mark.parametrize("name", EDGES)
def test_edge_fixture_through_batch_kernel(batches, name):
    """pip's 0x0000 / 0xFFFF corners (packets carrying their own checksum, all-zero
    headers, an empty segment under an all-zero pseudo-header) through each
    batch kernel the bench runs, against pip's results (make_golden.EDGES)."""
    b = batches[name]
    w = next(x for x in ALL.values() if x.cfg == b["cfg"])
    n, fam = b["n"], b["family"]
    if w.ragged and b.get("layout") == "bytes":
        arena, lens16, tc, _ = engine.gen_packed_bytes(n, b["first"], b["seed"], b["hdr"])
    elif w.ragged:
        arena, lens16, tc, _ = engine.gen_packed(n, b["first"], b["seed"], b["hdr"])
    elif b["length"]:
        arena = torch.empty(n * b["stride"], dtype=torch.uint8, device=DEV)
        engine.gen_fixed(arena, b["stride"], b["length"], n, b["first"], b["seed"], b["hdr"])
    else:
        arena = torch.zeros(n * b["stride"], dtype=torch.uint8, device=DEV)
    for o, hx in b["patches"]:
        v = patch_bytes(hx)
        arena[o:o + len(v)] = torch.frombuffer(bytearray(v), dtype=torch.uint8).to(DEV)
    assert sha(arena.cpu().numpy()) == b["arena_sha256"]
    pseudo = None
    if fam:
        flows, _ = engine.gen_flows(fam, b["n_flows"], b["seed"], b["proto"])
        rec = 12 if fam == 4 else 36
        if b["zero_flows"]:
            flows.view(b["n_flows"], rec)[torch.tensor(b["zero_flows"], device=DEV), :rec - 4] = 0
        pseudo = engine.prepare_flows(fam, flows, b["n_flows"])
    if w.ragged and b.get("layout") == "bytes":
        out = engine.checksum_packed_bytes(arena, lens16, tc, n, pseudo, b["n_flows"], None, b["first"])
    elif w.ragged:
        out = engine.checksum_packed(arena, lens16, tc, n, pseudo, b["n_flows"], None, b["first"])
    else:
        out = engine.checksum_fixed(arena, b["stride"], b["length"], n, pseudo, b["n_flows"], None, b["first"])
    assert b["kernel"] in last_kernel(), last_kernel()
    outs = [out]
    if b.get("alt"):  # the other fixed-stride schedule on the same bytes
        engine.tune(alt_flat_schedule=True)
        try:
            outs.append(engine.checksum_fixed(arena, b["stride"], b["length"], n, pseudo, b["n_flows"], None,
                                              b["first"]))
            assert b["alt"] in last_kernel(), last_kernel()
        finally:
            engine.tune()
    if b["kernel"] == "k_small<" and not fam:  # IPv4 headers: also through k_hdr (batches >= 8M headers)
        engine.tune(loads_per_lane=32)
        try:
            outs.append(engine.checksum_fixed(arena, b["stride"], b["length"], n, None, b["n_flows"], None, b["first"]))
            assert "k_hdr<" in last_kernel()
        finally:
            engine.tune()
    for out in outs:
        got = u16(out)
        assert int((got == 0).sum()) == b["n_zero"] and int((got == 0xFFFF).sum()) == b["n_ffff"]
        assert list(got[:16]) == b["head"]
        assert sha(got.astype("<u2")) == b["results_sha256"]


@pytest.mark.parametrize("small_k_log", [0, 1, 2, 3, 4])
def test_small_kernel_depth_leaves_other_kernels_exact(oracle, small_k_log):
    """Regression: the small kernel's packets-per-lane tune bits
    (24..27) once overlapped the flat kernel's loads-only probe bit, so a valid
    small_k_log silently broke k_flat.  Every kernel must stay exact under every
    documented small-kernel depth."""
    engine.tune(small_k_log=small_k_log)
    try:
        for w, n in ((CFG2, 300), (CFG3, 40), (CFG5, 40), (CFG1, 5000)):
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            pseudo = _pseudo(w)
            got = u16(engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 0))
            host = arena.cpu().numpy()
            want = oracle.batch_fixed(host, w.stride, w.length, n, w.family, w.proto, w.seed, N_FLOWS, 0)
            assert np.array_equal(got, want), (w.name, small_k_log)
    finally:
        engine.tune()


def test_device_flows_match_oracle(oracle):
    for fam, proto in ((4, 6), (6, 17)):
        seed = 0x1234 + fam
        flows, pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)
        want = oracle.flows_table(fam, seed, N_FLOWS, proto)
        assert flows.cpu().numpy().tobytes() == want
        # pseudo base from a host-uploaded table equals the device-generated one
        t = engine.flows_to_device(fam, want)
        assert torch.equal(engine.prepare_flows(fam, t, N_FLOWS), pseudo)


# ----------------------------------------------------------------------------
# 3. fixed-stride kernel: every launch shape, lengths, strides, alignments
# ----------------------------------------------------------------------------
LENGTHS = [0, 1, 2, 3, 15, 16, 17, 20, 31, 33, 64, 100, 1023, 1024, 1025, 1480, 4095, 8960, 8980, 9216, 9217,
           20001, 65535]


@pytest.mark.parametrize("lanes", [0, 1, 2, 4, 8, 16, 32, 64, 256])  # 256: k_wave, one packet per wave
def test_fixed_every_shape_vs_oracle(oracle, lanes):
    rng = np.random.default_rng(100 + lanes)
    engine.tune(lanes)
    try:
        for length in LENGTHS:
            for fam in (0, 4, 6):
                stride = int(rng.choice([length, (length + 7) // 8 * 8, (length + 15) // 16 * 16 + 16, length + 1]))
                stride = max(stride, 1)
                n = int(rng.integers(1, 40)) if length > 9000 else int(rng.integers(60, 300))
                misalign = int(rng.integers(0, 16))
                host = rng.integers(0, 256, n * stride, dtype=np.uint8)
                if rng.random() < 0.3:  # sprinkle all-0xFF / all-zero packets
                    host[:stride] = 0xFF
                    host[-stride:] = 0
                _, arena = upload(host, misalign)
                seed, proto, origin = int(rng.integers(0, 2**63)), int(rng.integers(0, 256)), int(rng.integers(0, 5000))
                pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
                out = engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin)
                if lanes == 256:
                    assert "k_wave<" in last_kernel()
                want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
                got = u16(out)
                assert np.array_equal(got, want), (lanes, length, stride, fam, misalign,
                                                   np.nonzero(got != want)[0][:5])
    finally:
        engine.tune()


@pytest.mark.parametrize("rows", [2, 4, 8, 16, 3, 5, 9, 13, 17, 25, 33])
@pytest.mark.parametrize("nt", [False, True])
@pytest.mark.parametrize("xcd", [False, True])
def test_flat_stream_kernel_vs_oracle(oracle, rows, nt, xcd):
    """The flat-stream fixed kernel (16-byte-multiple strides >= 1 KiB, aligned
    arena): packet boundaries at every lane position of a row, boundaries that
    fall exactly on row ends, stride padding wider than a row, runs cut short."""
    rng = np.random.default_rng(rows * 10 + nt + 100 * xcd)
    cases = [(1024, 1024), (1024, 1023), (1024, 0), (1040, 1025), (1488, 1480), (1504, 1480), (2048, 17),
             (3072, 2049), (8960, 8960), (8992, 8980), (9216, 8980), (65536, 65535)]
    try:
        for stride, length in cases:
            for blocks in (0, 1, 7, 9, 17):  # < 8 blocks: one group; 9/17: uneven XCD groups
                # k_flat itself at every stride (the default from 1 KiB to 64 KiB is k_flat_coop,
                # except at exactly 1 and 2 KiB)
                engine.tune(0, rows, blocks, plain_loads=not nt, nt_loads=nt, xcd_groups=xcd,
                            alt_flat_schedule=stride not in (1024, 2048))
                n = int(rng.integers(1, 20)) if stride > 20000 else int(rng.integers(1, 400))
                host = rng.integers(0, 256, n * stride, dtype=np.uint8)
                if n > 2:
                    host[stride:2 * stride] = 0xFF
                _, arena = upload(host, 0)
                fam = int(rng.choice([0, 4, 6]))
                seed, proto, origin = int(rng.integers(0, 2**62)), 6, int(rng.integers(0, 3000))
                pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
                got = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin))
                assert "k_flat<" in last_kernel()
                want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
                assert np.array_equal(got, want), (stride, length, n, blocks, np.nonzero(got != want)[0][:5])
                ok = engine.verify_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin).cpu().numpy()
                # a packet verifies exactly when its recomputed checksum is 0x0000
                assert np.array_equal(ok.astype(bool), got == 0)
    finally:
        engine.tune()


@pytest.mark.parametrize("ring", [17, 25, 33])
@pytest.mark.parametrize("rows", [0, 2, 48, 96])
def test_flat_coop_kernel_vs_oracle(oracle, ring, rows):
    """The block-cooperative flat stream (k_flat_coop, tune bit 28): a block's
    waves on interleaved rows of one task of K packets; boundaries at every
    lane, padding chunks, tasks cut short, tiny and large tasks."""
    rng = np.random.default_rng(ring * 100 + rows)
    cases = [(1024, 1024), (1024, 1023), (1024, 0), (1040, 1025), (1488, 1480), (1504, 1480), (2048, 17),
             (3072, 2049), (8960, 8960), (8992, 8980), (9216, 8980), (65536, 65535)]
    try:
        for stride, length in cases:
            # the coop stream is the default from 1 KiB to 64 KiB, except at exactly 1 and 2 KiB
            engine.tune(0, ring, 0, rows_per_task=rows, alt_flat_schedule=stride in (1024, 2048))
            n = int(rng.integers(1, 20)) if stride > 20000 else int(rng.integers(1, 700))
            host = rng.integers(0, 256, n * stride, dtype=np.uint8)
            if n > 2:
                host[stride:2 * stride] = 0xFF
            if n > 3:
                host[3 * stride:4 * stride] = 0  # all zero: 0xFFFF without a pseudo-header
            _, arena = upload(host, 0)
            fam = int(rng.choice([0, 4, 6]))
            seed, proto, origin = int(rng.integers(0, 2**62)), 6, int(rng.integers(0, 3000))
            pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
            got = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin))
            assert "k_flat_coop<" in last_kernel()
            want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
            assert np.array_equal(got, want), (stride, length, n, np.nonzero(got != want)[0][:5])
            if n > 3 and not fam:
                assert got[3] == 0xFFFF  # pip's ~fold(0) (pip_checksum.cpp:29-38)
            ok = engine.verify_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin).cpu().numpy()
            assert np.array_equal(ok.astype(bool), got == 0)
    finally:
        engine.tune()


@pytest.mark.parametrize("ring,rows,nt", [(0, 0, True), (4, 4, True), (16, 64, True), (8, 2, False), (16, 8, True)])
def test_tiny_stride_flat_kernel_vs_oracle(oracle, ring, rows, nt):
    """k_flat_tiny (8-byte-multiple strides 8..64 B, 16-byte-aligned arena;
    forced on for batches without pseudo-headers too; rings of 4/8/16 rows,
    tasks of 2..64 rows in whole LDS groups; strides up to 128 B reach the
    other fixed kernels): every stride, lengths 1 / 20 / stride-1 / stride and
    random ones, batch sizes around the task size, one task per wave and a
    capped grid that loops, implicit and explicit flows, RX verify, results
    aligned (vector stores) and shifted by one element (scalar stores)."""
    rng = np.random.default_rng(900 + rows + ring)
    try:
        for stride in range(8, 129, 8):
            hpp = stride // 8
            odd, pow2 = hpp, 1
            while odd % 2 == 0:
                odd, pow2 = odd // 2, pow2 * 2
            G = odd * max(1, pow2 // 2)  # rows per LDS group (tiny_group_rows)
            P = G * 128 // hpp
            run = max(1, min(2048 // P, (rows or 12) // G)) * P  # mirrors launch_fixed
            lengths = sorted({1, min(20, stride), stride - 1 or 1, stride, int(rng.integers(1, stride + 1))})
            for length in lengths:
                n = int(rng.choice([1, 2, run - 1, run, run + 1, 3 * run + 5, 20000]))
                blocks = int(rng.choice([0, 0, 1, 7]))
                engine.tune(0, ring, blocks, plain_loads=not nt, nt_loads=nt, rows_per_task=rows,
                            force_flat_tiny=True)
                fam = int(rng.choice([0, 4, 6]))
                host = rng.integers(0, 256, n * stride, dtype=np.uint8)
                if n > 3:
                    host[stride:2 * stride] = 0xFF
                    host[2 * stride:3 * stride] = 0
                _, arena = upload(host, 0)
                seed, proto, origin = int(rng.integers(0, 2**62)), 6, int(rng.integers(0, 3000))
                pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
                want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
                # results 8-/4-byte aligned (vector stores) or shifted by one element (scalar stores)
                shift = int(rng.integers(0, 2))
                out = torch.empty(n + 1, dtype=torch.int16, device=DEV)[shift:shift + n]
                okb = torch.empty(n + 1, dtype=torch.uint8, device=DEV)[shift:shift + n]
                got = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin, out=out))
                assert np.array_equal(got, want), (stride, length, n, blocks, shift, np.nonzero(got != want)[0][:5])
                ok = engine.verify_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin, ok=okb)
                assert np.array_equal(ok.cpu().numpy().astype(bool), got == 0)
        # explicit per-packet flow indices on the cfg1 shape
        n, L = 5003, 20
        host = rng.integers(0, 256, n * 24, dtype=np.uint8)
        _, arena = upload(host, 0)
        _, pseudo = engine.gen_flows(6, N_FLOWS, 77, 17)
        flow_of = rng.integers(0, N_FLOWS, n).astype(np.int32)
        engine.tune(0, ring, 0, plain_loads=not nt, nt_loads=nt, rows_per_task=rows, force_flat_tiny=True)
        got = u16(engine.checksum_fixed(arena, 24, L, n, pseudo, N_FLOWS, torch.from_numpy(flow_of).to(DEV), 0))
        engine.tune(flat_tiny=False)
        ref = u16(engine.checksum_fixed(arena, 24, L, n, pseudo, N_FLOWS, torch.from_numpy(flow_of).to(DEV), 0))
        assert np.array_equal(got, ref)
        for i in range(0, n, 11):
            s, d = oracle.flow6(77, int(flow_of[i]))
            assert got[i] == oracle.inet6_checksum(host[i * 24:i * 24 + L].tobytes(), 17, s, d)
    finally:
        engine.tune()


@pytest.mark.parametrize("misalign", [0, 1, 4, 8, 13])
def test_small_packet_kernel_vs_oracle(oracle, misalign):
    """k_small (one lane per packet, <= 64 bytes incl. the first chunk's offset):
    every length 0..49 at tight, odd, 8- and 16-aligned strides (and strides
    below 16), partial last tasks, implicit and explicit flows, RX verify; the
    same batches through k_fixed (small=False) must agree.  With a 16-byte
    aligned arena the 8-byte-multiple strides take k_flat_tiny by default, so
    k_small runs there with flat_tiny=False."""
    rng = np.random.default_rng(500 + misalign)
    try:
        for length in range(0, 50):
            for stride in sorted({max(length, 1), length + 1, length + 3, (length + 7) // 8 * 8 or 8,
                                  (length + 15) // 16 * 16 or 16, 24 if length <= 24 else length}):
                n = int(rng.choice([1, 255, 256, 257, 1000, 1500]))
                fam = int(rng.choice([0, 4, 6]))
                host = rng.integers(0, 256, n * stride + 16, dtype=np.uint8)
                if n > 3:
                    host[stride:2 * stride] = 0xFF
                    host[2 * stride:3 * stride] = 0
                _, arena = upload(host, misalign)
                seed, proto, origin = int(rng.integers(0, 2**62)), 17, int(rng.integers(0, 3000))
                pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
                want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
                engine.tune()
                got = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin))
                assert np.array_equal(got, want), (length, stride, n, fam, np.nonzero(got != want)[0][:5])
                ok = engine.verify_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin).cpu().numpy()
                assert np.array_equal(ok.astype(bool), got == 0)
                for arm in (dict(flat_tiny=False), dict(flat_tiny=False, small=False)):
                    engine.tune(**arm)
                    old = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin))
                    assert np.array_equal(old, want), (arm, length, stride, n)
        # explicit per-packet flow indices
        n, L = 3001, 20
        host = rng.integers(0, 256, n * 24, dtype=np.uint8)
        _, arena = upload(host, misalign)
        _, pseudo = engine.gen_flows(4, N_FLOWS, 99, 6)
        flow_of = rng.integers(0, N_FLOWS, n).astype(np.int32)
        engine.tune()
        got = u16(engine.checksum_fixed(arena, 24, L, n, pseudo, N_FLOWS, torch.from_numpy(flow_of).to(DEV), 0))
        for i in range(0, n, 7):
            s, d = oracle.flow4(99, int(flow_of[i]))
            assert got[i] == oracle.inet_checksum(host[i * 24:i * 24 + L].tobytes(), 6, s, d)
    finally:
        engine.tune()


@pytest.mark.parametrize("stride", [20, 24])
@pytest.mark.parametrize("ring,rows", [(32, 0), (8, 1), (16, 3), (24, 64), (16, 128),
                                       (33, 0), (9, 1), (17, 3), (25, 64), (17, 128)])
def test_header_row_kernel_vs_oracle(oracle, stride, ring, rows):
    """k_hdr (pipck_hdr.hip): packed 20/24-byte items with no pseudo-header
    (cfg1's IPv4 headers) streamed as rows of whole headers, each header split
    over two lanes.  Every length up to the stride (bytes past `len` masked,
    odd lengths), batches ending inside a row, on a row, on a wave-task and on
    a block-task boundary, all-0xFF / all-zero headers, RX verify; every ring
    and task size, one task per wave (ring 8/16/24/32) and the block-cooperative
    row order (9/17/25/33)."""
    rng = np.random.default_rng(700 + stride + ring + rows)
    engine.tune(0, ring, 0, rows_per_task=rows)
    try:
        per = (rows or 64) * (48 if stride == 20 else 42)  # headers per wave task
        for length in sorted({0, 1, 2, 3, 4, 5, 11, 19, 20, stride - 1, stride}):
            for n in sorted({1, 47, 48, 49, per - 1, per, per + 1, 4 * per - 1, 4 * per, 4 * per + 7, 20000}):
                host = rng.integers(0, 256, n * stride + 16, dtype=np.uint8)
                if n > 3:
                    host[stride:2 * stride] = 0xFF
                    host[2 * stride:3 * stride] = 0
                _, arena = upload(host, 0)
                want = oracle.batch_fixed(host, stride, length, n, 0, 0, 0, N_FLOWS, 0)
                got = u16(engine.checksum_fixed(arena, stride, length, n, None, N_FLOWS, None, 0))
                assert "k_hdr<" in last_kernel(), last_kernel()
                assert np.array_equal(got, want), (length, n, np.nonzero(got != want)[0][:5])
                ok = engine.verify_fixed(arena, stride, length, n, None, N_FLOWS, None, 0).cpu().numpy()
                assert "k_hdr<" in last_kernel()
                assert np.array_equal(ok.astype(bool), got == 0)
        # result arrays at every 2-byte / 1-byte offset from a 16-byte boundary (the
        # kernel writes 16-byte pieces only where the caller's array is aligned)
        n = 5000
        host = rng.integers(0, 256, n * stride + 16, dtype=np.uint8)
        _, arena = upload(host, 0)
        want = oracle.batch_fixed(host, stride, 20, n, 0, 0, 0, N_FLOWS, 0)
        for shift in range(8):
            buf = torch.zeros(n + 16, dtype=torch.int16, device=DEV)
            got = u16(engine.checksum_fixed(arena, stride, 20, n, None, N_FLOWS, None, 0, out=buf[shift:shift + n]))
            assert np.array_equal(got, want), shift
            assert not buf[:shift].any() and not buf[shift + n:].any(), shift  # nothing written outside
        okbuf = torch.zeros(n + 32, dtype=torch.uint8, device=DEV)
        for shift in (0, 1, 5, 15):
            okbuf.zero_()
            ok = engine.verify_fixed(arena, stride, 20, n, None, N_FLOWS, None, 0, ok=okbuf[shift:shift + n])
            assert np.array_equal(ok.cpu().numpy().astype(bool), want == 0) and not okbuf[:shift].any(), shift
        # checksummed IPv4 headers verify; one flipped bit is caught
        n = 5000
        host = rng.integers(0, 256, n * stride + 16, dtype=np.uint8)
        for i in range(n):
            host[i * stride + 10:i * stride + 12] = 0
            c = oracle.ip_checksum(host[i * stride:i * stride + 20].tobytes())
            host[i * stride + 10], host[i * stride + 11] = c >> 8, c & 0xFF
        host[17 * stride + 3] ^= 0x10
        _, arena = upload(host, 0)
        ok = engine.verify_fixed(arena, stride, 20, n, None, N_FLOWS, None, 0).cpu().numpy().astype(bool)
        assert not ok[17] and ok.sum() == n - 1
    finally:
        engine.tune()


@pytest.mark.parametrize("blocks", [0, 1, 9])
def test_short_stride_flat_kernel_vs_oracle(oracle, blocks):
    """k_flat_small (aligned arena, 16-byte-multiple strides below 1 KiB): many
    packet boundaries per row, padding chunks, empty packets, partial tasks,
    grid-stride tasks, RX verify, explicit flows; k_fixed/k_small (the
    fallback with flat_small=False) must agree."""
    rng = np.random.default_rng(900 + blocks)
    try:
        for stride in (16, 32, 48, 64, 80, 128, 144, 496, 512, 1008):  # < 64: the k_small fallback
            for length in sorted({0, 1, stride // 2 + 1, stride - 15, stride - 1, stride} - {-15}):
                if length < 0:
                    continue
                n = int(rng.choice([1, 63, 64, 65, 1000, 5000]))
                fam = int(rng.choice([0, 4, 6]))
                host = rng.integers(0, 256, n * stride, dtype=np.uint8)
                if n > 3:
                    host[stride:2 * stride] = 0xFF
                    host[2 * stride:3 * stride] = 0
                _, arena = upload(host, 0)
                seed, proto, origin = int(rng.integers(0, 2**62)), 6, int(rng.integers(0, 3000))
                pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
                want = oracle.batch_fixed(host, stride, length, n, fam, proto, seed, N_FLOWS, origin)
                engine.tune(blocks=blocks)
                got = u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin))
                assert np.array_equal(got, want), (stride, length, n, fam, np.nonzero(got != want)[0][:5])
                ok = engine.verify_fixed(arena, stride, length, n, pseudo, N_FLOWS, None, origin).cpu().numpy()
                assert np.array_equal(ok.astype(bool), got == 0)
                engine.tune(flat_small=False)
                assert np.array_equal(u16(engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, None,
                                                                origin)), want)
        n, stride = 2001, 96
        host = rng.integers(0, 256, n * stride, dtype=np.uint8)
        _, arena = upload(host, 0)
        _, pseudo = engine.gen_flows(6, N_FLOWS, 5, 17)
        flow_of = rng.integers(0, N_FLOWS, n).astype(np.int32)
        engine.tune(blocks=blocks)
        got = u16(engine.checksum_fixed(arena, stride, 90, n, pseudo, N_FLOWS, torch.from_numpy(flow_of).to(DEV), 0))
        for i in range(0, n, 11):
            s, d = oracle.flow6(5, int(flow_of[i]))
            assert got[i] == oracle.inet6_checksum(host[i * stride:i * stride + 90].tobytes(), 17, s, d)
    finally:
        engine.tune()


def test_fixed_grid_stride_loop(oracle):
    """Force a tiny grid so every block loops over many packets."""
    rng = np.random.default_rng(5)
    host = rng.integers(0, 256, 5000 * 1488, dtype=np.uint8)
    _, arena = upload(host)
    _, pseudo = engine.gen_flows(4, N_FLOWS, 77, 6)
    want = oracle.batch_fixed(host, 1488, 1480, 5000, 4, 6, 77, N_FLOWS, 123)
    for blocks in (1, 3, 17):
        engine.tune(blocks=blocks)
        try:
            got = u16(engine.checksum_fixed(arena, 1488, 1480, 5000, pseudo, N_FLOWS, None, 123))
        finally:
            engine.tune()
        assert np.array_equal(got, want), blocks


def test_fixed_explicit_flow_indices(oracle):
    rng = np.random.default_rng(6)
    n, L = 777, 333
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    _, arena = upload(host)
    flows, pseudo = engine.gen_flows(6, N_FLOWS, 99, 17)
    flow_of = rng.integers(0, N_FLOWS, n).astype(np.int32)
    got = u16(engine.checksum_fixed(arena, L, L, n, pseudo, N_FLOWS, torch.from_numpy(flow_of).to(DEV), 0))
    for i in range(n):
        s, d = oracle.flow6(99, int(flow_of[i]))
        assert got[i] == oracle.inet6_checksum(host[i * L:(i + 1) * L].tobytes(), 17, s, d)


# ----------------------------------------------------------------------------
# 4. ragged kernel and chains
# ----------------------------------------------------------------------------
def _ragged_case(rng, n, max_len=9000, gaps=True):
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[rng.random(n) < 0.1] = 0
    lens[rng.random(n) < 0.05] = 1
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 40)) if gaps else 0
        offs[i] = pos
        pos += int(lens[i])
    perm = rng.permutation(n)  # descriptors need not be in arena order
    return offs[perm], lens[perm], pos


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4099])
def test_ragged_vs_oracle(oracle, n):
    rng = np.random.default_rng(n)
    for fam, max_len in ((4, 9000), (6, 65535), (0, 300)):
        offs, lens, size = _ragged_case(rng, n, max_len)
        host = rng.integers(0, 256, size + 16, dtype=np.uint8)
        _, arena = upload(host, int(rng.integers(0, 16)))
        seed, proto, origin = 4242 + n, 6, int(rng.integers(0, 999))
        pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
        flows = (origin + np.arange(n)) % N_FLOWS
        desc = engine.make_desc(offs, lens, flows)
        got = u16(engine.checksum_ragged(arena, desc, pseudo))
        want = oracle.batch_ragged(host, offs, lens, fam, proto, seed, N_FLOWS, origin)
        assert np.array_equal(got, want), (fam, np.nonzero(got != want)[0][:5])
        ok = engine.verify_ragged(arena, desc, pseudo).cpu().numpy().astype(bool)
        assert np.array_equal(ok, got == 0)  # valid exactly when the recomputed checksum is 0x0000


@pytest.mark.parametrize("blocks", [1, 3, 8, 9, 17])
@pytest.mark.parametrize("xcd", [True, False])
@pytest.mark.parametrize("rows", [2, 4, 8, 3, 5, 9, 7, 13, 17, 25, 33])
@pytest.mark.parametrize("wide", [False, True])
def test_ragged_launch_shapes(oracle, blocks, xcd, rows, wide):
    """Every ragged row depth (plain and pipelined), 1- and 4-wave blocks, grids
    smaller and larger than the 8 XCD groups, tiles left over after the split."""
    rng = np.random.default_rng(blocks * 100 + rows * 2 + xcd)
    n = 64 * 23 + 5
    offs, lens, size = _ragged_case(rng, n, 3000)
    host = rng.integers(0, 256, size + 16, dtype=np.uint8)
    _, arena = upload(host, 0)
    _, pseudo = engine.gen_flows(4, N_FLOWS, 7, 6)
    desc = engine.make_desc(offs, lens, np.arange(n) % N_FLOWS)
    engine.tune(0, rows, blocks, xcd_groups=xcd, wide_blocks=wide)
    try:
        got = u16(engine.checksum_ragged(arena, desc, pseudo))
    finally:
        engine.tune()
    assert np.array_equal(got, oracle.batch_ragged(host, offs, lens, 4, 6, 7, N_FLOWS, 0))


def _packed_case(rng, n, max_len=3000):
    """Segments back to back at 16-byte granularity (packed tiles), with some
    tiles broken on purpose: a 16-byte gap, a misaligned tile, empty and odd
    segments.  Padding bytes are random, so tail masking is exercised."""
    lens = rng.integers(0, max_len + 1, n).astype(np.uint32)
    lens[rng.random(n) < 0.05] = 0
    lens[rng.random(n) < 0.2] |= 1
    offs = np.zeros(n, dtype=np.uint64)
    pos = 16
    for i in range(n):
        tile = i // 64
        if tile % 5 == 3 and i % 64 == 17:
            pos += 16                      # a gap: tile not packed
        if tile % 7 == 4 and i % 64 == 0:
            pos += 1                       # a misaligned tile: not packed
        elif i % 64 == 0:
            pos = (pos + 15) & ~15
        offs[i] = pos
        pos += (int(lens[i]) + 15) & ~15 if tile % 7 != 4 else int(lens[i])
    return offs, lens, pos + 16


@pytest.mark.parametrize("rows", [4, 8, 3, 5, 9, 7, 13, 17, 25, 33])
def test_ragged_packed_tiles(oracle, rows):
    rng = np.random.default_rng(rows)
    n = 64 * 40 + 9
    offs, lens, size = _packed_case(rng, n)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    _, arena = upload(host, 0)
    _, pseudo = engine.gen_flows(4, N_FLOWS, 7, 6)
    desc = engine.make_desc(offs, lens, np.arange(n) % N_FLOWS)
    want = oracle.batch_ragged(host, offs, lens, 4, 6, 7, N_FLOWS, 0)
    try:
        for packed in (True, False):
            engine.tune(0, rows, packed_tiles=packed)
            got = u16(engine.checksum_ragged(arena, desc, pseudo))
            assert np.array_equal(got, want), f"packed_tiles={packed}"
    finally:
        engine.tune()


def _packed_lens(rng, shape, n, oracle=None):
    if shape == "zipf":
        return oracle.zipf_lengths(4242, int(rng.integers(0, 1 << 30)), n)
    lens = {
        "uniform": lambda: rng.integers(0, 9001, n),
        "tiny": lambda: rng.integers(0, 33, n),          # every tile <= 2 chunks: lane-per-packet path
        "short": lambda: rng.integers(0, 120, n),        # many segment ends per row: the LDS-mark path
        "mixed": lambda: np.where(rng.random(n) < 0.5, rng.integers(0, 80, n), rng.integers(0, 4000, n)),
        "jumbo": lambda: rng.integers(30000, 65536, n),
        "edge": lambda: rng.choice([0, 1, 2, 15, 16, 17, 31, 32, 33, 1023, 1024, 1025, 65534, 65535], n),
    }[shape]()
    return np.asarray(lens, dtype=np.uint32)


def _packed_upload(rng, lens, misalign_padding=True):
    """Host + device arena in the packed layout (padding bytes random, so every
    tail mask matters); returns (host, offsets, arena, lens16, tile_chunk)."""
    chunks = (lens.astype(np.uint64) + 15) // 16
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(chunks)[:-1] * 16
    host = rng.integers(0, 256, int(chunks.sum()) * 16 + 16, dtype=np.uint8)
    _, arena = upload(host, 0)
    lens16 = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(DEV)
    tc = engine.packed_index(lens16)
    want_tc = np.concatenate([[0], np.cumsum(chunks)])[::64]
    got_tc = tc.cpu().numpy()
    assert np.array_equal(got_tc[:-1], want_tc[:len(got_tc) - 1]) and got_tc[-1] == chunks.sum()
    return host, offs, arena, lens16, tc


@pytest.mark.parametrize("shape", ["zipf", "uniform", "tiny", "short", "mixed", "jumbo", "edge"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 3001])
def test_packed_vs_oracle(oracle, shape, n):
    """pipck_checksum_packed / pipck_verify_packed (lengths + a per-64 index,
    no descriptors) against pip's algorithm, with implicit flows from an
    origin, explicit flow indices and no pseudo-header; both mixed-row paths
    (LDS marks, k_packed's default, and the scalar end loop: tune bit 19)."""
    rng = np.random.default_rng(hash((shape, n)) % 2**32)
    lens = _packed_lens(rng, shape, n, oracle)
    host, offs, arena, lens16, tc = _packed_upload(rng, lens)
    for fam, explicit in ((4, False), (6, True), (0, False)):
        seed, proto, origin = 99 + n, 6 if fam == 4 else 17, int(rng.integers(0, 1 << 40))
        pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
        flow_idx = (origin + np.arange(n)) % N_FLOWS
        flow_of = None
        if explicit:
            flow_idx = rng.integers(0, N_FLOWS, n)
            flow_of = torch.from_numpy(flow_idx.astype(np.int32)).to(DEV)
        if fam == 0:
            want = np.array([oracle.ip_checksum(host[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)],
                            dtype=np.uint16)
        elif explicit:
            want = np.array([oracle.inet6_checksum(host[int(o):int(o) + int(L)].tobytes(), proto,
                                                   *oracle.flow6(seed, int(f)), int(L))
                             for o, L, f in zip(offs, lens, flow_idx)], dtype=np.uint16)
        else:
            want = oracle.batch_ragged(host, offs, lens, fam, proto, seed, N_FLOWS, origin)
        for marks in (False, True):
            engine.tune(packed_marks_only=marks)
            try:
                got = u16(engine.checksum_packed(arena, lens16, tc, n, pseudo, N_FLOWS, flow_of,
                                                 0 if explicit else origin))
                ok = engine.verify_packed(arena, lens16, tc, n, pseudo, N_FLOWS, flow_of,
                                          0 if explicit else origin).cpu().numpy().astype(bool)
            finally:
                engine.tune()
            assert np.array_equal(got, want), (fam, marks, np.nonzero(got != want)[0][:5])
            assert np.array_equal(ok, got == 0)


@pytest.mark.parametrize("ring", [17, 25, 33])
@pytest.mark.parametrize("nt", [False, True])
def test_packed_rings_and_load_policy(oracle, ring, nt):
    rng = np.random.default_rng(ring * 2 + nt)
    n = 64 * 50 + 3
    lens = _packed_lens(rng, "mixed", n)
    host, offs, arena, lens16, tc = _packed_upload(rng, lens)
    _, pseudo = engine.gen_flows(4, N_FLOWS, 5, 6)
    engine.tune(0, ring, plain_loads=not nt, nt_loads=nt)
    try:
        got = u16(engine.checksum_packed(arena, lens16, tc, n, pseudo, N_FLOWS, None, 7))
    finally:
        engine.tune()
    assert np.array_equal(got, oracle.batch_ragged(host, offs, lens, 4, 6, 5, N_FLOWS, 7))


def test_packed_argument_checks():
    lens16 = torch.zeros(10, dtype=torch.int16, device=DEV)
    tc = engine.packed_index(lens16)
    arena = torch.zeros(64, dtype=torch.uint8, device=DEV)
    lib = _lib.load()
    out = torch.empty(10, dtype=torch.int16, device=DEV)
    rc = lib.pipck_checksum_packed(C.c_void_p(arena.data_ptr() + 1), C.c_void_p(lens16.data_ptr()),
                                   C.c_void_p(tc.data_ptr()), 10, None, 1, None, 0, C.c_void_p(out.data_ptr()), None)
    assert rc == _lib.PIPCK_EINVAL  # misaligned arena
    with pytest.raises(ValueError):  # the index says more bytes than the arena holds
        big = torch.full((10,), 100, dtype=torch.int16, device=DEV)
        engine.checksum_packed(arena, big, engine.packed_index(big))


@pytest.mark.parametrize("misalign", [0, 3, 8])
def test_ragged_tiny_segment_tiles(oracle, misalign):
    """Tiles whose segments all span <= 2 chunks take the lane-per-segment path
    (20-B IPv4 headers): tiles of 0..16-byte segments at 16-byte slots (plus
    the arena misalignment), tiles of 0..49 bytes at random offsets (chunk
    stream), long segments; the chunk stream alone (tiny_tiles=False) must agree."""
    rng = np.random.default_rng(70 + misalign)
    n = 64 * 30 + 17
    lens = rng.integers(0, 50, n).astype(np.uint32)
    tiny = np.arange(n) < 64 * 12  # first 12 tiles: every segment fits 2 chunks
    lens[tiny] = rng.integers(0, 17, int(tiny.sum()))
    lens[64 * 5:64 * 5 + 3] = 16
    lens[64 * 20:64 * 21] = rng.integers(0, 3000, 64)  # a tile with long segments
    lens[64 * 22 + 3] = 65535
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos = (pos + 15) // 16 * 16 if tiny[i] else pos + int(rng.integers(0, 20))
        offs[i] = pos
        pos += int(lens[i])
    host = rng.integers(0, 256, pos + 64, dtype=np.uint8)
    _, arena = upload(host, misalign)
    _, pseudo = engine.gen_flows(4, N_FLOWS, 11, 6)
    desc = engine.make_desc(offs, lens, np.arange(n) % N_FLOWS)
    want = oracle.batch_ragged(host, offs, lens, 4, 6, 11, N_FLOWS, 0)
    try:
        for tiny in (True, False):
            engine.tune(tiny_tiles=tiny)
            got = u16(engine.checksum_ragged(arena, desc, pseudo))
            assert np.array_equal(got, want), (tiny, np.nonzero(got != want)[0][:5])
            ok = engine.verify_ragged(arena, desc, pseudo).cpu().numpy().astype(bool)
            assert np.array_equal(ok, got == 0)
    finally:
        engine.tune()


@pytest.mark.parametrize("nl", [0, 2, 16])
def test_wave_per_packet_arm_ragged_vs_oracle(oracle, nl):
    """k_wave (pipck_wave.hip, the north_star's one-packet-per-wavefront shape,
    a measurement arm behind tune lanes_per_packet=256) on descriptor batches:
    unaligned, permuted, empty and 65,535-byte segments, several passes per
    packet (nl 2 = 2 KiB per pass), RX verify."""
    rng = np.random.default_rng(300 + nl)
    engine.tune(256, nl)
    try:
        for fam, max_len in ((4, 9000), (6, 65535), (0, 300)):
            n = int(rng.integers(500, 1500))
            offs, lens, size = _ragged_case(rng, n, max_len)
            host = rng.integers(0, 256, size + 16, dtype=np.uint8)
            _, arena = upload(host, int(rng.integers(0, 16)))
            seed, proto, origin = 77 + nl, 17, int(rng.integers(0, 999))
            pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
            desc = engine.make_desc(offs, lens, (origin + np.arange(n)) % N_FLOWS)
            got = u16(engine.checksum_ragged(arena, desc, pseudo))
            assert "k_wave<" in last_kernel()
            want = oracle.batch_ragged(host, offs, lens, fam, proto, seed, N_FLOWS, origin)
            assert np.array_equal(got, want), (fam, np.nonzero(got != want)[0][:5])
            ok = engine.verify_ragged(arena, desc, pseudo).cpu().numpy().astype(bool)
            assert np.array_equal(ok, got == 0)
        # out of the batch domain: 0 and PIPCK_ERANGE, as k_ragged
        offs = np.array([0, 10, 100_000, 5], dtype=np.uint64)
        lens = np.array([100, 70_000, 33, 0], dtype=np.uint32)
        host = rng.integers(0, 256, 200_000, dtype=np.uint8)
        _, arena = upload(host)
        err = torch.zeros(1, dtype=torch.int32, device=DEV)
        got = u16(engine.checksum_ragged(arena, engine.make_desc(offs, lens, np.zeros(4)), None, err=err))
        assert int(err.item()) & (1 << _lib.PIPCK_ERANGE) and got[1] == 0
        for i in (0, 2, 3):
            assert got[i] == oracle.ip_checksum(host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
    finally:
        engine.tune()


def test_ragged_out_of_domain_flags_error(oracle):
    rng = np.random.default_rng(9)
    host = rng.integers(0, 256, 200_000, dtype=np.uint8)
    _, arena = upload(host)
    offs = np.array([0, 10, 100_000, 5], dtype=np.uint64)
    lens = np.array([100, 70_000, 33, 0], dtype=np.uint32)
    desc = engine.make_desc(offs, lens, np.zeros(4))
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = u16(engine.checksum_ragged(arena, desc, None, err=err))
    assert int(err.item()) & (1 << _lib.PIPCK_ERANGE)
    assert got[1] == 0
    for i in (0, 2, 3):
        assert got[i] == oracle.ip_checksum(host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())


@pytest.mark.parametrize("fam", [4, 6])
def test_chains_vs_oracle(oracle, fam):
    """pip_inet{,6}_checksum_buf: odd-length middle segments restart byte pairing."""
    rng = np.random.default_rng(fam)
    n_pk = 700
    seg_lens, seg_begin = [], [0]
    for _ in range(n_pk):
        k = int(rng.integers(0, 7))
        seg_lens += [int(rng.choice([rng.integers(0, 9), rng.integers(0, 3000), 20, 8])) for _ in range(k)]
        seg_begin.append(len(seg_lens))
    seg_lens = np.array(seg_lens, dtype=np.uint32)
    offs = np.zeros(len(seg_lens), dtype=np.uint64)
    pos = 0
    for i, L in enumerate(seg_lens):
        pos += int(rng.integers(0, 17))
        offs[i] = pos
        pos += int(L)
    host = rng.integers(0, 256, pos + 16, dtype=np.uint8)
    _, arena = upload(host, 3)
    seed, proto = 31337, 17
    flows, pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)
    pkt_flow = rng.integers(0, N_FLOWS, n_pk).astype(np.int32)
    segs = engine.make_desc(offs, seg_lens, np.zeros(len(seg_lens)))
    got = u16(engine.checksum_chains(arena, segs, torch.tensor(seg_begin, dtype=torch.int64, device=DEV),
                                     torch.from_numpy(pkt_flow).to(DEV), pseudo))
    for p in range(n_pk):
        chain = [host[int(offs[s]):int(offs[s]) + int(seg_lens[s])].tobytes() for s in range(seg_begin[p], seg_begin[p + 1])]
        s, d = (oracle.flow4 if fam == 4 else oracle.flow6)(seed, int(pkt_flow[p]))
        fn = oracle.inet_checksum_chain if fam == 4 else oracle.inet6_checksum_chain
        assert got[p] == fn(chain, proto, s, d), p


def _chain_kats(kat, fn):
    from tests.golden.make_golden import pattern_bytes

    out = []
    for c in kat:
        if c["fn"] == fn:
            segs = [pattern_bytes(x) for x in c["segs"]]
            out.append((segs, c["proto"], bytes.fromhex(c["src"]), bytes.fromhex(c["dst"]), c["expect"]))
    return out


@pytest.mark.parametrize("fam", [4, 6])
def test_chain_known_answers_through_the_batch_chain_abi(kat, fam):
    """Every pip_inet{,6}_checksum_buf known answer (pip's compiled results, kat.json)
    through pipck_checksum_chains_n, each chain its own packet with its own flow --
    including the chains whose total_len passes 65,535 (2 x 40,000, 3 x 30,001 odd,
    65,535 + 1, 4 x 65,535, all-0xFF 4 x 65,535), where pip's pseudo-header gets a
    non-zero hi16(total_len) (pip/pip_checksum.cpp:105-107, 139-141).  Segments
    sit at odd and even arena offsets."""
    cases = _chain_kats(kat, "inet_chain" if fam == 4 else "inet6_chain")
    assert sum(1 for c in cases if sum(len(x) for x in c[0]) > 65535) >= 5
    rng = np.random.default_rng(fam * 7)
    blob, offs, lens, seg_begin, flows = bytearray(), [], [], [0], bytearray()
    for segs, proto, src, dst, _ in cases:
        for sg in segs:
            blob += bytes(int(rng.integers(0, 4)))  # odd / even starts
            offs.append(len(blob))
            lens.append(len(sg))
            blob += sg
        seg_begin.append(len(offs))
        flows += src + dst + bytes([proto]) + bytes(3)  # pipck_flow4 / pipck_flow6 record
    host = np.frombuffer(bytes(blob) + bytes(16), dtype=np.uint8)
    _, arena = upload(host, 5)
    pseudo = engine.prepare_flows(fam, engine.flows_to_device(fam, bytes(flows)), len(cases))
    segs_d = engine.make_desc(np.array(offs, dtype=np.uint64), np.array(lens, dtype=np.uint32), np.zeros(len(offs)))
    pkt_flow = torch.arange(len(cases), dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = u16(engine.checksum_chains(arena, segs_d, torch.tensor(seg_begin, dtype=torch.int64, device=DEV), pkt_flow,
                                     pseudo, err=err))
    assert int(err.item()) == 0
    want = np.array([c[4] for c in cases], dtype=np.uint16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), [len(x) for x in cases[i][0]], int(want[i]), int(got[i])) for i in bad[:5]]


@pytest.mark.parametrize("in_place", [True, False])
def test_chain_known_answers_through_the_tx_queue(kat, in_place):
    """The same known answers (v4 and v6 chains, the > 65,535-B totals among them)
    through the deferred TX queue (pipck_txq_add4 / add6 + flush): each field gets
    htons() of pip's own result, in place and with the copy path."""
    lib = _lib.load()
    ctx, q = C.c_void_p(), C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    _lib.check("pipck_txq_create", lib.pipck_txq_create(ctx, C.byref(q)))
    if not in_place:
        _lib.check("pipck_txq_inplace_max", lib.pipck_txq_inplace_max(q, 0))
    cases = [(4, c) for c in _chain_kats(kat, "inet_chain")] + [(6, c) for c in _chain_kats(kat, "inet6_chain")]
    fields = (C.c_uint8 * (2 * len(cases)))()
    keep = []
    try:
        for i, (fam, (segs, proto, src, dst, _)) in enumerate(cases):
            arr = (_lib.HSeg * max(len(segs), 1))()
            for j, sg in enumerate(segs):
                b = C.create_string_buffer(sg, max(len(sg), 1))
                keep.append(b)
                arr[j].ptr = C.cast(b, C.c_void_p)
                arr[j].len = len(sg)
            field = C.c_void_p(C.addressof(fields) + 2 * i)
            if fam == 4:
                _lib.check("add4", lib.pipck_txq_add4(q, arr, len(segs), proto, int.from_bytes(src, "little"),
                                                      int.from_bytes(dst, "little"), field))
            else:
                _lib.check("add6", lib.pipck_txq_add6(q, arr, len(segs), proto, src, dst, field))
        _lib.check("pipck_txq_flush", lib.pipck_txq_flush(q))
        got = np.frombuffer(bytes(fields), dtype=">u2")
        want = np.array([c[4] for _, c in cases], dtype=np.uint16)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(i), [len(x) for x in cases[i][1][0]], int(want[i]), int(got[i])) for i in bad[:5]]
    finally:
        lib.pipck_txq_destroy(q)
        lib.pipck_ctx_destroy(ctx)


# ----------------------------------------------------------------------------
# 5. RX verification kernel
# ----------------------------------------------------------------------------
def test_verify_fixed_accepts_checksummed_and_rejects_corrupted():
    w = CFG2
    n = 20000
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, 6)
    out = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)
    _insert_fixed(arena, w.stride, n, 16, out)
    ok = engine.verify_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)
    assert bool((ok == 1).all())
    rows = arena.view(n, w.stride)
    rows[::7, 100] ^= 0x5A
    ok = engine.verify_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS).cpu().numpy()
    assert not ok[::7].any() and ok[np.arange(n) % 7 != 0].all()


def _insert_fixed(arena, stride, n, field, out):
    """Store each result big-endian (htons) into its packet's checksum field."""
    rows = arena.view(n, stride)
    v = out.to(torch.int32) & 0xFFFF
    rows[:, field] = (v >> 8).to(torch.uint8)
    rows[:, field + 1] = (v & 0xFF).to(torch.uint8)


# ----------------------------------------------------------------------------
# 6. host-memory pipeline (H2D -> kernel -> D2H, two streams)
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline_vs_oracle(oracle, pinned):
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    try:
        w = CFG3
        n = 9000  # > one 64 MiB chunk: exercises double buffering
        host = oracle.gen_fixed_batch(w.seed, 0, n, w.length, w.hdr, w.stride, 8)
        flows = oracle.flows_table(6, w.seed, N_FLOWS, w.proto)
        out = np.zeros(n, dtype=np.uint16)
        src = host
        pin = None
        if pinned:
            pin = lib.pipck_host_alloc(host.size)
            C.memmove(pin, host.ctypes.data, host.size)
            src_ptr = C.c_void_p(pin)
        else:
            src_ptr = C.c_void_p(src.ctypes.data)
        fl = C.create_string_buffer(flows, len(flows))
        _lib.check("pipck_host_checksum_fixed",
                   lib.pipck_host_checksum_fixed(ctx, src_ptr, w.stride, w.length, n, 6, fl, N_FLOWS, 0,
                                                 C.c_void_p(out.ctypes.data)))
        if pin:
            lib.pipck_host_free(pin)
        want = oracle.batch_fixed(host, w.stride, w.length, n, 6, w.proto, w.seed, N_FLOWS, 0, 8)
        assert np.array_equal(out, want)
    finally:
        lib.pipck_ctx_destroy(ctx)


@pytest.mark.parametrize("shape", ["zipf_pinned", "zipf_pageable", "tiny_many", "after_fixed"])
def test_host_packed_bytes_pipeline_vs_oracle(oracle, shape):
    """pipck_host_checksum_packed_bytes: a byte-packed ragged batch in host
    memory (cfg4's shape, packets back to back) through ~64 MiB chunks of whole
    packets on two streams -- more than one chunk by bytes (Zipf) and by packet
    count (1.2M packets of 0-40 bytes) -- against the oracle; and after the
    fixed-stride pipeline sized the same context's buffers for 20-byte packets."""
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    pin = None
    try:
        w = CFG4
        if shape == "tiny_many":
            n = 1_200_000
            rng = np.random.default_rng(3)
            lens = rng.integers(0, 41, n).astype(np.uint32)
            offs = np.zeros(n, dtype=np.uint64)
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
            arena = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
        else:
            n = 150_000
            arena, offs, lens = oracle.gen_packed_bytes_batch(w.seed, 0, n, w.hdr)
        if shape == "after_fixed":
            hdrs = oracle.gen_fixed_batch(CFG1.seed, 0, 4 << 20, 20, CFG1.hdr, 20, 8)
            tmp = np.zeros(4 << 20, dtype=np.uint16)
            _lib.check("pipck_host_checksum_fixed", lib.pipck_host_checksum_fixed(
                ctx, C.c_void_p(hdrs.ctypes.data), 20, 20, 4 << 20, 0, None, 0, 0, C.c_void_p(tmp.ctypes.data)))
            assert np.array_equal(tmp[:5000], oracle.batch_fixed(hdrs, 20, 20, 5000, 0, 0, 0, 1, 0))
        flows = oracle.flows_table(4, w.seed, N_FLOWS, w.proto)
        lens16 = lens.astype(np.uint16)
        out = np.zeros(n, dtype=np.uint16)
        if shape == "zipf_pinned":
            pin = lib.pipck_host_alloc(arena.size)
            C.memmove(pin, arena.ctypes.data, arena.size)
            src = C.c_void_p(pin)
        else:
            src = C.c_void_p(arena.ctypes.data)
        fl = C.create_string_buffer(flows, len(flows))
        _lib.check("pipck_host_checksum_packed_bytes", lib.pipck_host_checksum_packed_bytes(
            ctx, src, C.c_void_p(lens16.ctypes.data), n, 4, fl, N_FLOWS, 7, C.c_void_p(out.ctypes.data)))
        want = oracle.batch_ragged(arena, offs, lens, 4, w.proto, w.seed, N_FLOWS, 7, 8)
        assert np.array_equal(out, want), np.nonzero(out != want)[0][:5]
    finally:
        if pin:
            lib.pipck_host_free(pin)
        lib.pipck_ctx_destroy(ctx)


# ----------------------------------------------------------------------------
# 7. generator shard invariance
# ----------------------------------------------------------------------------
def test_generator_is_shard_invariant():
    w = CFG5
    whole = torch.empty(1000 * w.stride, dtype=torch.uint8, device=DEV)
    part = torch.empty(400 * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(whole, w.stride, w.length, 1000, 5_000_000, w.seed, w.hdr)
    engine.gen_fixed(part, w.stride, w.length, 400, 5_000_300, w.seed, w.hdr)
    assert torch.equal(whole[300 * w.stride:700 * w.stride], part)


# ----------------------------------------------------------------------------
# 8. full BASELINE.json sizes: sampled oracle comparison + checksum-of-checksum
# ----------------------------------------------------------------------------
# cfg1 also at 256M headers: the size the f3 line is profiled at, where k_hdr runs
FULL = [(CFG1, 1 << 20, 0), (CFG1, 256 << 20, 3), (CFG2, 4 << 20, 0), (CFG3, 1 << 20, 0), (CFG5, 8 << 20, 8 << 20)]
FIELD = {1: 10, 2: 16, 3: 6, 4: 16, 5: 16}  # ip_sum / th_sum / uh_sum offsets


@pytest.mark.parametrize("w,n,first", FULL, ids=[f"{w.name}_{n}" for w, n, _ in FULL])
def test_full_size_fixed(oracle, w, n, first):
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, first, w.seed, w.hdr)
    pseudo = _pseudo(w)
    out = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, first)
    if w.cfg == 1:
        assert ("k_hdr<5," if n >= 8 << 20 else "k_small<") in last_kernel()
    got = u16(out)
    rng = np.random.default_rng(w.cfg)
    for i in rng.choice(n, 1500, replace=False):
        pkt = oracle.packet(w.seed, first + int(i), w.length, w.hdr)
        f = (first + int(i)) % N_FLOWS
        if w.family == 4:
            want = oracle.inet_checksum(pkt, w.proto, *oracle.flow4(w.seed, f))
        elif w.family == 6:
            want = oracle.inet6_checksum(pkt, w.proto, *oracle.flow6(w.seed, f))
        else:
            want = oracle.ip_checksum(pkt)
        assert got[i] == want, (w.name, int(i))
    _insert_fixed(arena, w.stride, n, FIELD[w.cfg], out)
    again = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, first)
    assert int((again != 0).sum().item()) == 0
    ok = engine.verify_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, first)
    assert bool((ok == 1).all())
    del arena, out, again, ok
    torch.cuda.empty_cache()


BULK = [(CFG1, 1 << 20, 0, "k_small<"), (CFG1, 256 << 20, 3, "k_hdr<5,"), (CFG2, 4 << 20, 0, "k_flat_coop<32,"),
        (CFG3, 1 << 20, 0, "k_flat_coop<32,"), (CFG5, 8 << 20, 8 << 20, "k_flat_coop<32,")]


@pytest.mark.parametrize("w,n,first,kernel", BULK, ids=[f"{w.name}_{n}" for w, n, _, _ in BULK])
def test_full_batch_bit_exact_with_pip(w, n, first, kernel):
    """Each fixed-stride BASELINE batch in bulk: every packet
    -- cfg5's 8M of rank 1's shard (ids 8M..16M, 75 GB), cfg2's 4M, cfg3's 1M,
    cfg1's 1M headers and 256M (f3's size) -- checksummed on the GPU by the
    bench kernel, then every result compared with pip's own compiled
    pip_inet{,6}_checksum / pip_ip_checksum (oracle/_ref; the oracle's
    restatement where _ref is absent) over the same bytes, regenerated on the
    host in chunks -- not a sample."""
    import os

    from oracle.oracle import Oracle, Reference

    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, first, w.seed, w.hdr)
    out = engine.checksum_fixed(arena, w.stride, w.length, n, _pseudo(w), N_FLOWS, None, first)
    assert kernel in last_kernel()
    got = u16(out)
    del arena, out
    torch.cuda.empty_cache()
    orc = Oracle()
    ref = Reference() if Reference.available() else None
    flows = orc.flows_table(w.family, w.seed, N_FLOWS, w.proto)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    chunk = max(1 << 19, n >> 5)
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        host = orc.gen_fixed_batch(w.seed, first + c0, m, w.length, w.hdr, w.stride, threads)
        if ref is not None:
            want = ref.batch_fixed(host, w.stride, w.length, m, w.family, w.proto, flows, N_FLOWS, first + c0, threads)
        else:
            want = orc.batch_fixed(host, w.stride, w.length, m, w.family, w.proto, w.seed, N_FLOWS, first + c0, threads)
        bad = np.nonzero(got[c0:c0 + m] != want)[0]
        assert bad.size == 0, (c0, bad[:5])
        del host


def test_cfg4_full_batch_bit_exact_with_pip():
    """cfg4 in bulk, byte-packed as the bench runs it: all 8M Zipf packets
    checksummed by the bench kernel (k_packedb), then the arena's own bytes copied
    back in ~1M-packet pieces and every packet checksummed by pip's compiled
    pip_inet_checksum (oracle/_ref; the restatement where it is absent) at its
    byte offset -- not a sample."""
    import os

    from oracle.oracle import Oracle, Reference

    w, n = CFG4, 8 << 20
    arena, lens16, to, lens = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
    assert "k_packedb<" in last_kernel()
    got = u16(out)
    L = lens.cpu().numpy().astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(L.astype(np.uint64))[:-1]
    orc = Oracle()
    ref = Reference() if Reference.available() else None
    flows = orc.flows_table(4, w.seed, N_FLOWS, w.proto)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    chunk = 1 << 20
    for c0 in range(0, n, chunk):
        m = min(chunk, n - c0)
        b0, b1 = int(offs[c0]), int(offs[c0 + m - 1]) + int(L[c0 + m - 1])
        host = arena[b0:b1].cpu().numpy()
        o = offs[c0:c0 + m] - np.uint64(b0)
        if ref is not None:
            want = ref.batch_ragged(host, o, L[c0:c0 + m], 4, w.proto, flows, N_FLOWS, c0, threads)
        else:
            want = orc.batch_ragged(host, o, L[c0:c0 + m], 4, w.proto, w.seed, N_FLOWS, c0, threads)
        bad = np.nonzero(got[c0:c0 + m] != want)[0]
        assert bad.size == 0, (c0, bad[:5])
        del host
    del arena, out
    torch.cuda.empty_cache()


def test_full_size_ragged(oracle):
    w, n = CFG4, 8 << 20
    arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_ragged(arena, desc, pseudo)
    got = u16(out)
    d = desc.cpu().numpy()
    offs = d[:, 0].astype(np.uint64)
    L = (d[:, 1] & 0xFFFFFFFF).astype(np.uint32)
    assert 900 < L.mean() < 1080
    rng = np.random.default_rng(4)
    for i in rng.choice(n, 1500, replace=False):
        assert L[i] == oracle.zipf_len(w.seed, int(i))
        pkt = oracle.packet(w.seed, int(i), int(L[i]), w.hdr)
        assert got[i] == oracle.inet_checksum(pkt, w.proto, *oracle.flow4(w.seed, int(i) % N_FLOWS)), int(i)
    # checksum-of-checksum over the whole ragged batch
    o = torch.from_numpy(offs.astype(np.int64)).to(DEV) + 16
    v = out.to(torch.int32) & 0xFFFF
    arena[o] = (v >> 8).to(torch.uint8)
    arena[o + 1] = (v & 0xFF).to(torch.uint8)
    again = engine.checksum_ragged(arena, desc, pseudo)
    assert int((again != 0).sum().item()) == 0
    assert bool((engine.verify_ragged(arena, desc, pseudo) == 1).all())
    arena[o[::5] + 2] ^= 0x41  # corrupt every fifth packet's destination port
    ok = engine.verify_ragged(arena, desc, pseudo).cpu().numpy()
    assert not ok[::5].any() and ok[np.arange(n) % 5 != 0].all()
    del arena, desc, out, again
    torch.cuda.empty_cache()


def test_full_size_packed(oracle):
    """cfg4 at its BASELINE size through the packed-lengths ABI (the bench's
    path): equal to the descriptor kernel on the same arena, sampled against
    the oracle, and checksum-of-checksum over the whole batch."""
    w, n = CFG4, 8 << 20
    arena, lens16, tc, lens = engine.gen_packed(n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_packed(arena, lens16, tc, n, pseudo, N_FLOWS, None, 0)
    got = u16(out)
    L = lens.cpu().numpy().astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum((L.astype(np.uint64) + 15) // 16)[:-1] * 16
    desc = engine.make_desc(offs, L, np.arange(n) % N_FLOWS)
    assert np.array_equal(got, u16(engine.checksum_ragged(arena, desc, pseudo)))
    del desc
    rng = np.random.default_rng(44)
    for i in rng.choice(n, 1500, replace=False):
        pkt = oracle.packet(w.seed, int(i), int(L[i]), w.hdr)
        assert got[i] == oracle.inet_checksum(pkt, w.proto, *oracle.flow4(w.seed, int(i) % N_FLOWS)), int(i)
    o = torch.from_numpy(offs.astype(np.int64)).to(DEV) + 16
    v = out.to(torch.int32) & 0xFFFF
    arena[o] = (v >> 8).to(torch.uint8)
    arena[o + 1] = (v & 0xFF).to(torch.uint8)
    again = engine.checksum_packed(arena, lens16, tc, n, pseudo, N_FLOWS, None, 0)
    assert int((again != 0).sum().item()) == 0
    assert bool((engine.verify_packed(arena, lens16, tc, n, pseudo, N_FLOWS, None, 0) == 1).all())
    del arena, out, again
    torch.cuda.empty_cache()


# ----------------------------------------------------------------------------
# 8b. byte-packed ragged batches (pipck_checksum_packed_bytes: cfg4's bench layout)
# ----------------------------------------------------------------------------
def _packedb_upload(rng, lens, lead=0):
    """Host + device arena in the byte-packed layout (packets back to back, no
    padding; `lead` random bytes before packet 0 via a shifted index is not
    possible -- the index starts at 0 -- so the arena itself is 128-B aligned
    and the first tile starts on a line); bytes after the last packet up to the
    16-B boundary are random too.  Returns (host, offsets, arena, lens16, tile_off)."""
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(lens.astype(np.uint64))[:-1]
    total = int(lens.astype(np.uint64).sum())
    host = rng.integers(0, 256, (total + 15) // 16 * 16 + 16, dtype=np.uint8)
    _, arena = upload(host, 0)
    lens16 = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).to(DEV)
    to = engine.packed_bytes_index(lens16)
    want = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))])[::64]
    got = to.cpu().numpy()
    assert np.array_equal(got[:-1], want[:len(got) - 1]) and got[-1] == total
    return host, offs, arena, lens16, to


PACKEDB_SHAPES = {1: 32, 4: 48, 8: 0}  # waves per tile -> tune loads_per_lane (0: the default, 8 waves, ring 3)


@pytest.mark.parametrize("tile_waves", [1, 4, 8])
@pytest.mark.parametrize("shape", ["zipf", "uniform", "tiny", "short", "mixed", "jumbo", "edge", "sixteen"])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 3001])
def test_packed_bytes_vs_oracle(oracle, shape, n, tile_waves):
    """Byte-packed batches: segments at every byte alignment (odd starts swap
    pip's byte pairing), chunks split between two segments, rows wholly inside
    one segment, tiles with a segment under 16 bytes (lane-per-segment path),
    empty segments; implicit / explicit flows and no pseudo-header; RX verify.
    tile_waves: the waves of k_packedb's block streaming one tile (rows dealt
    round-robin): 8 (the default, a ring of 3), 4 (tune loads_per_lane 48, a
    ring of 8), 1 (loads_per_lane 32, a ring of 32)."""
    engine.tune(loads_per_lane=PACKEDB_SHAPES[tile_waves])
    try:
        _packed_bytes_vs_oracle(oracle, shape, n, "k_packedb<")
        assert last_kernel().split("(")[0].endswith(f", {tile_waves}>")
    finally:
        engine.tune()


def _packed_bytes_vs_oracle(oracle, shape, n, kname):
    rng = np.random.default_rng(hash(("b", shape, n)) % 2**32)
    if shape == "sixteen":  # the smallest lengths the chunk stream takes
        lens = rng.choice([16, 17, 18, 31, 32, 33, 47], n).astype(np.uint32)
    else:
        lens = _packed_lens(rng, shape, n, oracle)
    host, offs, arena, lens16, to = _packedb_upload(rng, lens)
    for fam, explicit in ((4, False), (6, True), (0, False)):
        seed, proto, origin = 77 + n, 6 if fam == 4 else 17, int(rng.integers(0, 1 << 40))
        pseudo = engine.gen_flows(fam, N_FLOWS, seed, proto)[1] if fam else None
        flow_of = None
        flow_idx = (origin + np.arange(n)) % N_FLOWS
        if explicit:
            flow_idx = rng.integers(0, N_FLOWS, n)
            flow_of = torch.from_numpy(flow_idx.astype(np.int32)).to(DEV)
        if fam == 0:
            want = np.array([oracle.ip_checksum(host[int(o):int(o) + int(L)].tobytes()) for o, L in zip(offs, lens)],
                            dtype=np.uint16)
        elif explicit:
            want = np.array([oracle.inet6_checksum(host[int(o):int(o) + int(L)].tobytes(), proto,
                                                   *oracle.flow6(seed, int(f)), int(L))
                             for o, L, f in zip(offs, lens, flow_idx)], dtype=np.uint16)
        else:
            want = oracle.batch_ragged(host, offs, lens, fam, proto, seed, N_FLOWS, origin)
        got = u16(engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, flow_of,
                                               0 if explicit else origin))
        assert kname in last_kernel()
        ok = engine.verify_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, flow_of,
                                        0 if explicit else origin).cpu().numpy().astype(bool)
        assert np.array_equal(got, want), (fam, np.nonzero(got != want)[0][:5])
        assert np.array_equal(ok, got == 0)


def test_packed_bytes_equals_packed_on_the_same_packets(oracle):
    """The byte-packed and the 16-B-granular layouts of one Zipf batch give the
    same results (device generators: same packet bytes, different padding)."""
    w, n = CFG4, 200_003
    a16, l16, tc, lens = engine.gen_packed(n, 5, w.seed, w.hdr)
    ab, lb, to, lens_b = engine.gen_packed_bytes(n, 5, w.seed, w.hdr)
    assert torch.equal(lens, lens_b)
    assert ab.numel() == (int(lens.to(torch.int64).sum().item()) + 15) // 16 * 16
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    x = engine.checksum_packed(a16, l16, tc, n, pseudo, N_FLOWS, None, 5)
    y = engine.checksum_packed_bytes(ab, lb, to, n, pseudo, N_FLOWS, None, 5)
    assert torch.equal(x, y)
    host, offs, hl = oracle.gen_packed_bytes_batch(w.seed, 5, 3000, w.hdr)
    assert np.array_equal(ab[:len(host)].cpu().numpy()[:int(offs[-1] + hl[-1])], host[:int(offs[-1] + hl[-1])])


def test_packedb_shapes_agree_full_size():
    """cfg4's 8M Zipf batch: k_packedb at every block width and ring depth the
    launcher has (tune loads_per_lane 32 = one wave, a ring of 32; 48 = 4 waves,
    a ring of 8; 72 / 0 / 74 = 8 waves, rings of 2 / 3 (the default) / 4) gives
    the same results, checksums and verify both."""
    w, n = CFG4, 8 << 20
    arena, lens16, to, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    engine.tune(loads_per_lane=32)
    try:
        want = engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
    finally:
        engine.tune()
    shapes = {32: "32, true, 1>", 48: "8, true, 4>", 72: "2, true, 8>", 0: "3, true, 8>", 74: "4, true, 8>"}
    for lq, tail in shapes.items():
        engine.tune(loads_per_lane=lq)
        try:
            got = engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
            assert last_kernel().split("(")[0].endswith(tail), (lq, last_kernel())
            ok = engine.verify_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
        finally:
            engine.tune()
        assert torch.equal(got, want), lq
        assert torch.equal(ok.to(torch.bool), want == 0), lq
    del arena


def test_packed_bytes_argument_checks():
    lens16 = torch.full((10,), 20, dtype=torch.int16, device=DEV)
    to = engine.packed_bytes_index(lens16)
    arena = torch.zeros(512, dtype=torch.uint8, device=DEV)
    lib = _lib.load()
    out = torch.empty(10, dtype=torch.int16, device=DEV)
    rc = lib.pipck_checksum_packed_bytes(C.c_void_p(arena.data_ptr() + 16), C.c_void_p(lens16.data_ptr()),
                                         C.c_void_p(to.data_ptr()), 10, None, 1, None, 0,
                                         C.c_void_p(out.data_ptr()), None)
    assert rc == _lib.PIPCK_EINVAL  # not 128-byte aligned
    with pytest.raises(ValueError):  # the index says more bytes than the arena holds
        big = torch.full((10,), 100, dtype=torch.int16, device=DEV)
        engine.checksum_packed_bytes(arena[:960 - 512], big, engine.packed_bytes_index(big))


def test_full_size_packed_bytes(oracle):
    """cfg4 at its BASELINE size in the byte-packed layout (the bench's path):
    equal to the descriptor kernel on the same packets, sampled against the
    oracle, and checksum-of-checksum over the whole batch."""
    w, n = CFG4, 8 << 20
    arena, lens16, to, lens = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
    got = u16(out)
    L = lens.cpu().numpy().astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(L.astype(np.uint64))[:-1]
    desc = engine.make_desc(offs, L, np.arange(n) % N_FLOWS)
    assert np.array_equal(got, u16(engine.checksum_ragged(arena, desc, pseudo)))
    del desc
    rng = np.random.default_rng(45)
    for i in rng.choice(n, 1500, replace=False):
        pkt = oracle.packet(w.seed, int(i), int(L[i]), w.hdr)
        assert got[i] == oracle.inet_checksum(pkt, w.proto, *oracle.flow4(w.seed, int(i) % N_FLOWS)), int(i)
    o = torch.from_numpy(offs.astype(np.int64)).to(DEV) + 16
    v = out.to(torch.int32) & 0xFFFF
    arena[o] = (v >> 8).to(torch.uint8)
    arena[o + 1] = (v & 0xFF).to(torch.uint8)
    again = engine.checksum_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0)
    assert int((again != 0).sum().item()) == 0
    assert bool((engine.verify_packed_bytes(arena, lens16, to, n, pseudo, N_FLOWS, None, 0) == 1).all())
    del arena, out, again
    torch.cuda.empty_cache()


# ----------------------------------------------------------------------------
# 9. deferred TX queue: mixed v4/v6 chains + IPv4 headers
# ----------------------------------------------------------------------------
@pytest.mark.parametrize("in_place", [True, False])
def test_txq_mixed_batches_vs_oracle(oracle, in_place):
    """in_place: small flushes read the pinned staging in place (default);
    False forces the H2D / D2H copy path that large flushes take."""
    lib = _lib.load()
    ctx, q = C.c_void_p(), C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    _lib.check("pipck_txq_create", lib.pipck_txq_create(ctx, C.byref(q)))
    if not in_place:  # per queue: every flush takes the copies
        _lib.check("pipck_txq_inplace_max", lib.pipck_txq_inplace_max(q, 0))
    rng = np.random.default_rng(99)
    try:
        for n_pk in (1, 300, 5000):  # the queue is reused and grows
            fields = (C.c_uint8 * (2 * n_pk))()
            keep, want = [], []
            for i in range(n_pk):
                kind = int(rng.integers(0, 3))
                field = C.c_void_p(C.addressof(fields) + 2 * i)
                if kind == 2:  # IPv4 header, ip_sum = 0
                    hdr = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
                    hdr[10:12] = b"\0\0"
                    buf = C.create_string_buffer(bytes(hdr), 20)
                    keep.append(buf)
                    _lib.check("add_ip", lib.pipck_txq_add_ip(q, buf, 20, field))
                    want.append(oracle.ip_checksum(bytes(hdr)))
                    continue
                segs = [rng.integers(0, 256, int(rng.choice([20, 8, rng.integers(0, 9), rng.integers(0, 9000)])),
                                     dtype=np.uint8).tobytes() for _ in range(int(rng.integers(1, 4)))]
                arr = (_lib.HSeg * len(segs))()
                for j, sgm in enumerate(segs):
                    b = C.create_string_buffer(sgm, max(len(sgm), 1))
                    keep.append(b)
                    arr[j].ptr = C.cast(b, C.c_void_p)
                    arr[j].len = len(sgm)
                proto = int(rng.choice([6, 17]))
                if kind == 0:
                    s, d = rng.bytes(4), rng.bytes(4)
                    _lib.check("add4", lib.pipck_txq_add4(q, arr, len(segs), proto, int.from_bytes(s, "little"),
                                                          int.from_bytes(d, "little"), field))
                    want.append(oracle.inet_checksum_chain(segs, proto, s, d))
                else:
                    s, d = rng.bytes(16), rng.bytes(16)
                    _lib.check("add6", lib.pipck_txq_add6(q, arr, len(segs), proto, s, d, field))
                    want.append(oracle.inet6_checksum_chain(segs, proto, s, d))
            assert lib.pipck_txq_pending(q) == n_pk
            _lib.check("pipck_txq_flush", lib.pipck_txq_flush(q))
            assert lib.pipck_txq_pending(q) == 0
            got = np.frombuffer(bytes(fields), dtype=">u2")  # htons(result), as pip stores it
            assert np.array_equal(got, np.array(want, dtype=np.uint16)), n_pk
    finally:
        lib.pipck_txq_destroy(q)
        lib.pipck_ctx_destroy(ctx)


def test_txq_submit_complete_pipeline(oracle):
    """Double-buffered async flush: batches submitted while the next one fills,
    fields written at the following submit/complete; a reused queue; flush
    after submit; empty submits."""
    lib = _lib.load()
    ctx, q = C.c_void_p(), C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    _lib.check("pipck_txq_create", lib.pipck_txq_create(ctx, C.byref(q)))
    rng = np.random.default_rng(1234)
    try:
        _lib.check("empty submit", lib.pipck_txq_submit(q))
        _lib.check("empty complete", lib.pipck_txq_complete(q))
        n_batches, per = 7, 333
        fields = (C.c_uint8 * (2 * n_batches * per))()
        keep, want = [], []
        for bi in range(n_batches):
            for i in range(per):
                k = bi * per + i
                segs = [rng.integers(0, 256, 20, dtype=np.uint8).tobytes(),
                        rng.integers(0, 256, int(rng.integers(0, 3000)), dtype=np.uint8).tobytes()]
                arr = (_lib.HSeg * 2)()
                for j, sgm in enumerate(segs):
                    b = C.create_string_buffer(sgm, max(len(sgm), 1))
                    keep.append(b)
                    arr[j].ptr = C.cast(b, C.c_void_p)
                    arr[j].len = len(sgm)
                s, d = rng.bytes(4), rng.bytes(4)
                _lib.check("add4", lib.pipck_txq_add4(q, arr, 2, 6, int.from_bytes(s, "little"),
                                                      int.from_bytes(d, "little"),
                                                      C.c_void_p(C.addressof(fields) + 2 * k)))
                want.append(oracle.inet_checksum_chain(segs, 6, s, d))
            assert lib.pipck_txq_pending(q) == per
            if bi == 3:
                _lib.check("flush", lib.pipck_txq_flush(q))  # completes the in-flight batch and this one
                assert lib.pipck_txq_inflight(q) == 0
            else:
                _lib.check("submit", lib.pipck_txq_submit(q))
                assert lib.pipck_txq_pending(q) == 0 and lib.pipck_txq_inflight(q) == per
                # every batch before this one is already stored
                got = np.frombuffer(bytes(fields), dtype=">u2")[:bi * per]
                assert np.array_equal(got, np.array(want[:bi * per], dtype=np.uint16)), bi
        _lib.check("complete", lib.pipck_txq_complete(q))
        assert lib.pipck_txq_inflight(q) == 0
        got = np.frombuffer(bytes(fields), dtype=">u2")
        assert np.array_equal(got, np.array(want, dtype=np.uint16))
    finally:
        lib.pipck_txq_destroy(q)
        lib.pipck_ctx_destroy(ctx)


@pytest.mark.parametrize("in_place", [True, False])
@pytest.mark.parametrize("register", [False, True])
def test_txq_zero_copy_segments(oracle, register, in_place):
    """pipck_txq_add4_zc / add6_zc: segments read in place from pinned host
    memory (pipck_host_alloc, or a registered numpy buffer), mixed in one batch
    with staged chains and IPv4 headers; flushed and pipelined."""
    lib = _lib.load()
    ctx, q = C.c_void_p(), C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    _lib.check("pipck_txq_create", lib.pipck_txq_create(ctx, C.byref(q)))
    if not in_place:  # per queue: every flush takes the copies
        _lib.check("pipck_txq_inplace_max", lib.pipck_txq_inplace_max(q, 0))
    rng = np.random.default_rng(4321 + register)
    size = 4 << 20
    if register:
        host = np.zeros(size + 4096, dtype=np.uint8)
        off0 = (-host.ctypes.data) % 4096
        pool = host[off0:off0 + size]
        base = pool.ctypes.data
        _lib.check("pipck_host_register", lib.pipck_host_register(C.c_void_p(base), size))
    else:
        base = lib.pipck_host_alloc(size)
        assert base
        pool = np.ctypeslib.as_array((C.c_uint8 * size).from_address(base))
    try:
        # a segment outside every pinned range is refused, and nothing is queued
        plain = C.create_string_buffer(b"x" * 64, 64)
        bad = (_lib.HSeg * 1)()
        bad[0].ptr, bad[0].len = C.cast(plain, C.c_void_p), 64
        fld = (C.c_uint8 * 2)()
        assert lib.pipck_txq_add4_zc(q, bad, 1, 6, 1, 2, C.cast(fld, C.c_void_p)) == _lib.PIPCK_EINVAL
        bad[0].ptr, bad[0].len = C.c_void_p(base + size - 8), 64  # runs past the end of the range
        assert lib.pipck_txq_add4_zc(q, bad, 1, 6, 1, 2, C.cast(fld, C.c_void_p)) == _lib.PIPCK_EINVAL
        assert lib.pipck_txq_pending(q) == 0
        for rnd in range(2):
            n_pk = 700
            fields = (C.c_uint8 * (2 * n_pk))()
            keep, want, pos = [], [], 0
            for i in range(n_pk):
                field = C.c_void_p(C.addressof(fields) + 2 * i)
                kind = int(rng.integers(0, 4))
                segs = [rng.integers(0, 256, int(rng.choice([20, 32, rng.integers(0, 9), rng.integers(0, 3000)])),
                                     dtype=np.uint8).tobytes() for _ in range(int(rng.integers(1, 4)))]
                if kind == 3:  # IPv4 header (staged)
                    hdr = bytearray(rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
                    hdr[10:12] = b"\0\0"
                    b = C.create_string_buffer(bytes(hdr), 20)
                    keep.append(b)
                    _lib.check("add_ip", lib.pipck_txq_add_ip(q, b, 20, field))
                    want.append(oracle.ip_checksum(bytes(hdr)))
                    continue
                arr = (_lib.HSeg * len(segs))()
                for j, sgm in enumerate(segs):
                    if kind in (0, 1):  # zero-copy: bytes placed in the pinned pool at any alignment
                        pos += int(rng.integers(0, 16))
                        pool[pos:pos + len(sgm)] = np.frombuffer(sgm, dtype=np.uint8)
                        arr[j].ptr = C.c_void_p(base + pos)
                        pos += len(sgm)
                    else:
                        b = C.create_string_buffer(sgm, max(len(sgm), 1))
                        keep.append(b)
                        arr[j].ptr = C.cast(b, C.c_void_p)
                    arr[j].len = len(sgm)
                proto = int(rng.choice([6, 17]))
                if kind in (0, 2):
                    s, d = rng.bytes(4), rng.bytes(4)
                    fn = lib.pipck_txq_add4_zc if kind == 0 else lib.pipck_txq_add4
                    _lib.check("add4", fn(q, arr, len(segs), proto, int.from_bytes(s, "little"),
                                          int.from_bytes(d, "little"), field))
                    want.append(oracle.inet_checksum_chain(segs, proto, s, d))
                else:
                    s, d = rng.bytes(16), rng.bytes(16)
                    _lib.check("add6_zc", lib.pipck_txq_add6_zc(q, arr, len(segs), proto, s, d, field))
                    want.append(oracle.inet6_checksum_chain(segs, proto, s, d))
                if rnd == 1 and i % 100 == 99:
                    _lib.check("submit", lib.pipck_txq_submit(q))
            _lib.check("flush", lib.pipck_txq_flush(q))
            got = np.frombuffer(bytes(fields), dtype=">u2")
            assert np.array_equal(got, np.array(want, dtype=np.uint16)), (rnd, np.nonzero(got != want)[0][:5])
    finally:
        lib.pipck_txq_destroy(q)
        lib.pipck_ctx_destroy(ctx)
        if register:
            lib.pipck_host_unregister(C.c_void_p(base))
        else:
            lib.pipck_host_free(C.c_void_p(base))


@pytest.mark.parametrize("mode", ["api", "env_only"])
def test_txq_auto_zero_copy(oracle, mode, monkeypatch):
    """pipck_txq_auto_zero_copy: plain add4/add6 read pinned segments in place
    and copy the rest.  Shown by rewriting every source buffer after add and
    before flush: a pinned segment's checksum follows the new bytes, a copied
    one keeps the add-time bytes.  The mode is an explicit per-queue opt-in:
    PIPCK_TXQ_AUTO_ZERO_COPY in the environment alone changes nothing (every
    segment keeps its add-time bytes).  Chains of more than 32 segments are read
    in place segment by segment too.  A pinned range with queued in-place
    segments cannot be freed (PIPCK_EBUSY) until their batch completes; once
    freed, a zero-copy add of it is refused (never read in place)."""
    monkeypatch.setenv("PIPCK_TXQ_AUTO_ZERO_COPY", "1")
    auto = mode == "api"
    lib = _lib.load()
    ctx, q = C.c_void_p(), C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    _lib.check("pipck_txq_create", lib.pipck_txq_create(ctx, C.byref(q)))
    if auto:
        _lib.check("auto_zero_copy", lib.pipck_txq_auto_zero_copy(q, 1))
    size = 1 << 20
    base = lib.pipck_host_alloc(size)
    assert base
    pool = np.ctypeslib.as_array((C.c_uint8 * size).from_address(base))
    rng = np.random.default_rng(77 + auto)
    freed = False
    try:
        n_pk = 300
        fields = (C.c_uint8 * (2 * n_pk))()
        keep, finals, pos = [], [], 0
        for i in range(n_pk):
            field = C.c_void_p(C.addressof(fields) + 2 * i)
            nseg = 40 if i == 7 else int(rng.integers(1, 4))  # one chain longer than 32 segments
            arr = (_lib.HSeg * nseg)()
            segs_final = []
            for j in range(nseg):
                ln = int(rng.choice([0, 20, int(rng.integers(1, 1500))]))
                old = rng.integers(0, 256, ln, dtype=np.uint8)
                new = rng.integers(0, 256, ln, dtype=np.uint8)
                if rng.integers(0, 2) or (i == 7 and j >= 32):  # pinned
                    pos += int(rng.integers(0, 16))
                    pool[pos:pos + ln] = old
                    arr[j].ptr = C.c_void_p(base + pos)
                    keep.append(("pinned", pos, new))
                    pos += ln
                    # read at flush in auto mode -> the rewritten bytes count
                    segs_final.append(new.tobytes() if auto else old.tobytes())
                else:  # ordinary memory: copied at add -> the add-time bytes count
                    b = C.create_string_buffer(old.tobytes(), max(ln, 1))
                    arr[j].ptr = C.cast(b, C.c_void_p)
                    keep.append(("plain", b, new))
                    segs_final.append(old.tobytes())
                arr[j].len = ln
            proto = int(rng.choice([6, 17]))
            if i % 2:
                s_, d_ = rng.bytes(4), rng.bytes(4)
                _lib.check("add4", lib.pipck_txq_add4(q, arr, nseg, proto, int.from_bytes(s_, "little"),
                                                      int.from_bytes(d_, "little"), field))
                finals.append(oracle.inet_checksum_chain(segs_final, proto, s_, d_))
            else:
                s_, d_ = rng.bytes(16), rng.bytes(16)
                _lib.check("add6", lib.pipck_txq_add6(q, arr, nseg, proto, s_, d_, field))
                finals.append(oracle.inet6_checksum_chain(segs_final, proto, s_, d_))
        for kind, where, new in keep:  # rewrite every source after add
            if kind == "pinned":
                pool[where:where + len(new)] = new
            elif len(new):
                C.memmove(where, new.tobytes(), len(new))
        if auto:  # queued in-place segments hold the range
            assert lib.pipck_host_free(C.c_void_p(base)) == _lib.PIPCK_EBUSY
            assert b"in place" in lib.pipck_last_error()
        _lib.check("flush", lib.pipck_txq_flush(q))
        got = np.frombuffer(bytes(fields), dtype=">u2")
        assert np.array_equal(got, np.array(finals, dtype=np.uint16)), np.nonzero(got != finals)[0][:5]
        # submitted but not completed: still held
        seg = (_lib.HSeg * 1)()
        seg[0].ptr, seg[0].len = C.c_void_p(base + 64), 32
        fld = (C.c_uint8 * 2)()
        _lib.check("add4_zc", lib.pipck_txq_add4_zc(q, seg, 1, 6, 1, 2, C.cast(fld, C.c_void_p)))
        _lib.check("submit", lib.pipck_txq_submit(q))
        assert lib.pipck_host_free(C.c_void_p(base)) == _lib.PIPCK_EBUSY
        _lib.check("complete", lib.pipck_txq_complete(q))
        # completed: the range can go, and a freed range is never read in place again
        _lib.check("pipck_host_free", lib.pipck_host_free(C.c_void_p(base)))
        freed = True
        assert lib.pipck_txq_add4_zc(q, seg, 1, 6, 1, 2, C.cast(fld, C.c_void_p)) == _lib.PIPCK_EINVAL
        assert lib.pipck_txq_pending(q) == 0
    finally:
        lib.pipck_txq_destroy(q)
        lib.pipck_ctx_destroy(ctx)
        if not freed:
            lib.pipck_host_free(C.c_void_p(base))


@pytest.mark.parametrize("weights", [[64, 60, 62, 58, 64, 61, 63, 59], [1, 64, 2, 64, 3, 64, 4, 64], [7] * 8])
def test_flat_xcd_weighted_deal_same_results(oracle, weights):
    """k_flat_xw (the XCD-weighted static deal, pipck_tune_xcd_weights; VERDICT r03
    item 7): blocks an XCD does not keep exit at once and the kept ones take the
    tasks in dispatch order -- every packet is summed exactly once, results equal
    k_flat's and the oracle's, at cfg2's stride and at batch sizes around a period."""
    w = CFG2
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    for n in (4096 * 8 + 7, 200003, 1 << 20):
        arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
        engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
        engine.tune(alt_flat_schedule=True)  # k_flat (cfg2's default is k_flat_coop since round 4)
        try:
            want = u16(engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS))
            assert "k_flat<24," in last_kernel()
            engine.tune_xcd_weights(weights, max(weights))
            got = u16(engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS))
            assert "k_flat_xw<24," in last_kernel(), last_kernel()
        finally:
            engine.tune_xcd_weights(None, 0)
            engine.tune()
        assert np.array_equal(got, want), np.nonzero(got != want)[0][:5]
        host = arena[:2000 * w.stride].cpu().numpy()
        assert np.array_equal(got[:2000], oracle.batch_fixed(host, w.stride, w.length, 2000, 4, w.proto, w.seed,
                                                             N_FLOWS, 0))


def test_hdr_in_place_probe_stores_ip_sum(oracle):
    """k_hdr's measurement arm (tune bit 28): each header's
    checksum stored into its own ip_sum (htons, byte 10, as pip_netif.cpp:97
    stores it) instead of the result array -- every header then verifies."""
    w = CFG1
    n = (8 << 20) + 13
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    want = u16(engine.checksum_fixed(arena, w.stride, w.length, n))
    engine.tune(loads_per_lane=32, hdr_in_place=True)
    try:
        sentinel = torch.full((n,), 0x1234, dtype=torch.int16, device=DEV)
        engine.checksum_fixed(arena, w.stride, w.length, n, out=sentinel)
        assert "k_hdr<5," in last_kernel()
    finally:
        engine.tune()
    assert (sentinel == 0x1234).all()  # the result array is untouched
    h = arena.view(n, 20).cpu().numpy()
    stored = h[:, 10].astype(np.uint16) << 8 | h[:, 11]
    assert np.array_equal(stored, want)
    ok = engine.verify_fixed(arena, w.stride, w.length, n).cpu().numpy()
    assert ok.all()


def test_prepared_calls_equal_the_wrappers():
    """bench.py's step: the C-ABI call bound once (engine.prepare_checksum_fixed /
    prepare_checksum_packed_bytes) gives the wrappers' results, run after run,
    and a rebound output is written where the binding says."""
    w = CFG2
    n = 5000
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, 7, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    want = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 7)
    run, out = engine.prepare_checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 7)
    for _ in range(3):
        out.zero_()
        run()
        assert torch.equal(out, want)
    with pytest.raises(ValueError):  # the span check runs once, at binding
        engine.prepare_checksum_fixed(arena[:(n - 1) * w.stride + w.length - 1], w.stride, w.length, n)
    w4 = CFG4
    ab, lb, to, _ = engine.gen_packed_bytes(3001, 11, w4.seed, w4.hdr)
    _, p4 = engine.gen_flows(4, N_FLOWS, w4.seed, w4.proto)
    want = engine.checksum_packed_bytes(ab, lb, to, 3001, p4, N_FLOWS, None, 11)
    run, out = engine.prepare_checksum_packed_bytes(ab, lb, to, 3001, p4, N_FLOWS, None, 11)
    run()
    assert torch.equal(out, want)
    torch.cuda.synchronize()


def test_results_into_pinned_host_memory():
    """d_out / d_ok may point into pinned host memory (INTEGRATION.md §2,
    bench.py --results-host): the fixed-stride, byte-packed and verify kernels
    write there exactly what they write to HBM."""
    w = CFG2
    n = 20000
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, 3, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    want = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 3)
    host = torch.full((n,), -1, dtype=torch.int16, pin_memory=True)
    run, out = engine.prepare_checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 3, out=host)
    run()
    torch.cuda.synchronize()
    assert out.device.type == "cpu" and torch.equal(out, want.cpu())
    ok = torch.zeros(n, dtype=torch.uint8, pin_memory=True)
    engine.verify_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 3, ok=ok)
    torch.cuda.synchronize()
    assert torch.equal(ok.to(torch.bool), (want == 0).cpu())
    w4 = CFG4
    ab, lb, to, _ = engine.gen_packed_bytes(5000, 0, w4.seed, w4.hdr)
    _, p4 = engine.gen_flows(4, N_FLOWS, w4.seed, w4.proto)
    want = engine.checksum_packed_bytes(ab, lb, to, 5000, p4, N_FLOWS, None, 0)
    host = torch.full((5000,), -1, dtype=torch.int16, pin_memory=True)
    run, out = engine.prepare_checksum_packed_bytes(ab, lb, to, 5000, p4, N_FLOWS, None, 0, out=host)
    run()
    torch.cuda.synchronize()
    assert torch.equal(out, want.cpu())
