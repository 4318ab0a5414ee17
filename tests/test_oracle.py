"""CPU: the oracle (oracle/pipck_oracle.c) pinned against pip's own outputs.

The fixtures in tests/golden/ were produced by pip's real pip_checksum.cpp
(tests/golden/make_golden.py); these tests need no GPU and no /root/reference.
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import edge_inputs_cpu, oracle_edge_results, run_case
from pip_amd.workloads import ALL, N_FLOWS

EDGES = sorted(k for k in json.loads((Path(__file__).parent / "golden" / "batches.json").read_text())
               if k.startswith("edge_"))


def test_oracle_matches_every_known_answer(oracle, kat):
    bad = [(c["fn"], c["expect"], run_case(oracle, c)) for c in kat if run_case(oracle, c) != c["expect"]]
    assert not bad, bad[:5]


def test_survey_known_answers(oracle):
    # SURVEY.md section 8a / 8c, measured on the compiled reference
    assert oracle.ip_checksum(bytes(20)) == 0xFFFF
    assert oracle.ip_checksum(b"\xff\xff") == 0x0000
    assert oracle.standard_checksum(b"\xff\xff") == 0xFFFF
    assert oracle.ip_checksum(b"") == 0xFFFF
    assert oracle.ip_checksum(b"\x01\x02\x03") == 0xFBFD
    assert oracle.ip_checksum(bytes.fromhex("450000730000400040110000c0a80001c0a800c7")) == 0xB861
    ff = b"\xff" * 131076
    assert oracle.ip_checksum(ff[:131074]) == 0x0000
    assert oracle.ip_checksum(ff) == 0x0001  # u32 wrap: RFC 1071 would give 0x0000
    assert oracle.inet_checksum(b"", 6, bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])) == 0xEBF6
    assert oracle.inet_checksum(b"", 0, bytes(4), bytes(4)) == 0xFFFF
    assert oracle.inet_checksum(bytes.fromhex("deadbeef01"), 6, bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])) == 0x4D54
    assert oracle.standard_checksum(bytes.fromhex("deadbeef01"), None, 0x1234) == 0xB0D1
    v6 = lambda x: bytes([0xFD] + [0] * 14 + [x])  # noqa: E731
    assert oracle.inet6_checksum(bytes.fromhex("deadbeef01"), 17, v6(1), v6(2)) == 0x6747
    src, dst = bytes([192, 168, 33, 2]), bytes([192, 168, 33, 1])
    assert oracle.inet_checksum_chain([b"\x01\x02\x03", b"\x04\x05\x06"], 6, src, dst) == 0x2E98
    assert oracle.inet_checksum(bytes(range(1, 7)), 6, src, dst) == 0x3393


def test_even_chains_equal_flat(oracle):
    rng = np.random.default_rng(1)
    for _ in range(50):
        segs = [rng.integers(0, 256, 2 * int(rng.integers(0, 40)), dtype=np.uint8).tobytes() for _ in range(3)]
        segs.append(rng.integers(0, 256, int(rng.integers(0, 99)), dtype=np.uint8).tobytes())  # last may be odd
        flat = b"".join(segs)
        s, d = rng.bytes(4), rng.bytes(4)
        assert oracle.inet_checksum_chain(segs, 6, s, d) == oracle.inet_checksum(flat, 6, s, d)


@pytest.mark.parametrize("name", sorted(ALL))
def test_generator_and_batch_match_reference_fixture(oracle, batches, name):
    """The CPU generator twin reproduces the fixture arena byte-for-byte and the
    oracle reproduces pip's results over it."""
    import hashlib

    b, w = batches[name], ALL[name]
    if w.ragged:
        arena, offs, lens = oracle.gen_ragged_batch(b["seed"], b["first"], b["n"], b["hdr"])
        assert hashlib.sha256(lens.astype("<u4").tobytes()).hexdigest() == b["lengths_sha256"]
        out = oracle.batch_ragged(arena, offs, lens, b["family"], b["proto"], b["seed"], N_FLOWS, b["first"], 4)
    else:
        arena = oracle.gen_fixed_batch(b["seed"], b["first"], b["n"], b["length"], b["hdr"], b["stride"], 4)
        out = oracle.batch_fixed(arena, b["stride"], b["length"], b["n"], b["family"], b["proto"], b["seed"],
                                 N_FLOWS, b["first"], 4)
    assert hashlib.sha256(arena.tobytes()).hexdigest() == b["arena_sha256"]
    assert hashlib.sha256(out.astype("<u2").tobytes()).hexdigest() == b["results_sha256"]
    assert list(out[:16]) == b["head"]


def test_fixture_layouts_are_the_shipped_ones(batches):
    """The fixtures pin the layouts the product runs: cfg1 at the
    packed 20-B stride the bench uses, cfg4 as the packed (16-B granular)
    arena pipck_checksum_packed reads."""
    assert batches["cfg1_ipv4_header"]["stride"] == ALL["cfg1_ipv4_header"].stride == 20
    assert batches["cfg4_tcp4_zipf"]["stride"] == 0 and "lengths_sha256" in batches["cfg4_tcp4_zipf"]


@pytest.mark.parametrize("name", EDGES)
def test_oracle_reproduces_edge_fixture(oracle, batches, name):
    """Edge batches (pip's 0x0000 / 0xFFFF corners through the batch layouts):
    the CPU rebuild of the inputs matches pip's bytes and the oracle pip's results."""
    b = batches[name]
    arena, offs, lens, flows = edge_inputs_cpu(oracle, b)
    assert hashlib.sha256(arena.tobytes()).hexdigest() == b["arena_sha256"]
    out = oracle_edge_results(oracle, b, arena, offs, lens, flows)
    assert hashlib.sha256(out.astype("<u2").tobytes()).hexdigest() == b["results_sha256"]
    assert list(out[:16]) == b["head"]
    assert int((out == 0).sum()) == b["n_zero"] and int((out == 0xFFFF).sum()) == b["n_ffff"]


def test_edge_fixtures_cover_both_corners(batches):
    edges = [batches[k] for k in EDGES]
    assert sum(b["n_zero"] for b in edges) > 0 and sum(b["n_ffff"] for b in edges) > 0
    # 0xFFFF under a pseudo-header (total 0: empty segment, zero addresses, proto 0)
    assert any(b["family"] and b["n_ffff"] for b in edges)
    # and 0x0000 through every batch kernel family the bench runs
    kernels = {b["kernel"] for b in edges if b["n_zero"]} | {b["alt"] for b in edges if b["n_zero"] and b.get("alt")}
    assert {"k_flat<24,", "k_flat_coop<32,", "k_small<", "k_packed<", "k_packedb<"} <= kernels
    # and 0xFFFF (pip's ~fold(0), pip_checksum.cpp:29-38) through the jumbo and
    # byte-packed bench kernels, from all-zero packets with no pseudo-header
    ffff = {b["kernel"] for b in edges if b["n_ffff"] and not b["family"]} | \
        {b["alt"] for b in edges if b["n_ffff"] and not b["family"] and b.get("alt")}
    assert {"k_flat_coop<32,", "k_flat<32,", "k_packedb<", "k_small<"} <= ffff


def test_zipf_shape(oracle):
    lens = oracle.zipf_lengths(0x9E3779B97F4A7C15 ^ 4, 0, 20000)
    assert lens.min() >= 64 and lens.max() <= 9000
    # mean ~987 B, P(L<=128) ~0.49, P(L>=1460) ~0.19
    assert 900 < lens.mean() < 1080
    assert 0.46 < (lens <= 128).mean() < 0.52
    assert 0.16 < (lens >= 1460).mean() < 0.22


def test_generator_edge_classes(oracle):
    """0.1 % all-zero and 0.1 % all-0xFF packets exercise the 0x0000/0xFFFF edge."""
    seed = 0x9E3779B97F4A7C15 ^ 2
    cls = [oracle.packet(seed, i, 32, 1) for i in range(20000)]
    zero = sum(1 for p in cls if p == bytes(32))
    ones = sum(1 for p in cls if p[:16] == b"\xff" * 16)
    assert 5 <= zero <= 45 and 5 <= ones <= 45


def test_reference_cross_check_if_built(oracle):
    """Where pip's real code is built (oracle/_ref), random vectors agree."""
    from oracle.oracle import Reference

    if not Reference.available():
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    ref = Reference()
    rng = np.random.default_rng(7)
    for _ in range(300):
        n = int(rng.integers(0, 3000))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s0 = int(rng.integers(0, 2**32))
        assert oracle.standard_checksum(data, None, s0) == ref.standard_checksum(data, None, s0)
        a, b = rng.bytes(16), rng.bytes(16)
        p = int(rng.integers(0, 256))
        assert oracle.inet6_checksum(data, p, a, b) == ref.inet6_checksum(data, p, a, b)
        segs = [rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes() for _ in range(4)]
        assert oracle.inet_checksum_chain(segs, p, a[:4], b[:4]) == ref.inet_checksum_chain(segs, p, a[:4], b[:4])
