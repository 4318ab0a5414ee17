#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from pip's REAL checksum code.

Runs only in the build container, where /root/reference exists:
    make -C oracle ref          # compiles pip_checksum.cpp + pip's stack into oracle/_ref/
    python tests/golden/make_golden.py

Writes
  kat.json            known-answer vectors: inputs (hex or a byte pattern) and the
                      results of pip's own functions (pip/pip_checksum.cpp:9-148)
  batches.json        per BASELINE.json config, a reduced batch made by the
                      generator spec (oracle/pipck_oracle.c) in the layout the
                      product runs it in (cfg1 packed at a 20-B stride; cfg4's
                      arena is also the packed-lengths layout): sha256 of the
                      arena bytes, and sha256 + head of pip's results over it;
                      plus "edge_*" batches whose results include pip's 0x0000
                      and 0xFFFF corners (EDGES below), so the fold edge is pinned
                      through every batch kernel, not only through the KATs
  stack_replay.txt    every IP packet pip's real stack emits for the scripted
                      exchange in oracle/stack_replay.cpp (link-substitution test)

The oracle restatement is checked against pip on every vector while writing.
"""
from __future__ import annotations

import hashlib
import json
import random
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from oracle.oracle import Oracle, Reference  # noqa: E402
from pip_amd.workloads import ALL, N_FLOWS  # noqa: E402

OUT = Path(__file__).resolve().parent


def pattern_bytes(spec: dict) -> bytes:
    if "hex" in spec:
        return bytes.fromhex(spec["hex"])
    n = spec["len"]
    if spec["pattern"] == "const":
        return bytes([spec["byte"]]) * n
    if spec["pattern"] == "affine":  # (i * mul + add) & 0xFF
        i = np.arange(n, dtype=np.uint64)
        return ((i * spec["mul"] + spec["add"]) & 0xFF).astype(np.uint8).tobytes()
    raise ValueError(spec)


def kat_cases(rng: random.Random) -> list[dict]:
    C = []
    hx = lambda b: {"hex": bytes(b).hex()}  # noqa: E731
    ip = lambda s: bytes(int(x) for x in s.split("."))  # noqa: E731

    def v6(last):
        a = bytearray(16)
        a[0] = 0xFD
        a[15] = last
        return bytes(a)

    # SURVEY.md 8a/8c known answers
    C.append({"fn": "standard", "data": hx(b""), "sum": 0})
    C.append({"fn": "ip", "data": hx(b"")})
    C.append({"fn": "ip", "data": hx(bytes(20))})
    C.append({"fn": "ip", "data": hx(b"\xff\xff")})
    C.append({"fn": "standard", "data": hx(b"\xff\xff"), "sum": 0})
    C.append({"fn": "ip", "data": hx(b"\x01\x02\x03")})
    C.append({"fn": "ip", "data": hx(bytes.fromhex("450000730000400040110000c0a80001c0a800c7"))})
    for n in (131070, 131072, 131074, 131076, 131078, 200001):  # u32 wrap threshold
        C.append({"fn": "standard", "data": {"pattern": "const", "byte": 255, "len": n}, "sum": 0})
        C.append({"fn": "ip", "data": {"pattern": "const", "byte": 255, "len": n}})
    C.append({"fn": "standard", "data": {"pattern": "const", "byte": 255, "len": 70000}, "sum": 0xFFFFFFF0})
    C.append({"fn": "standard", "data": hx(bytes.fromhex("deadbeef01")), "sum": 0x1234})
    C.append({"fn": "inet", "data": hx(b""), "proto": 6, "src": ip("10.0.0.1").hex(), "dst": ip("10.0.0.2").hex()})
    C.append({"fn": "inet", "data": hx(b""), "proto": 0, "src": ip("0.0.0.0").hex(), "dst": ip("0.0.0.0").hex()})
    C.append({"fn": "inet", "data": hx(bytes.fromhex("deadbeef01")), "proto": 6,
              "src": ip("10.0.0.1").hex(), "dst": ip("10.0.0.2").hex()})
    C.append({"fn": "inet6", "data": hx(bytes.fromhex("deadbeef01")), "proto": 17,
              "src": v6(1).hex(), "dst": v6(2).hex()})
    C.append({"fn": "inet_chain", "segs": [hx(b"\x01\x02\x03"), hx(b"\x04\x05\x06")], "proto": 6,
              "src": ip("192.168.33.2").hex(), "dst": ip("192.168.33.1").hex()})
    for fam_fn, w in (("inet_chain", 4), ("inet6_chain", 16)):  # a chain of one empty pip_buf
        C.append({"fn": fam_fn, "segs": [], "proto": 17, "src": (b"\x6c\x54\x38\x75" * 4)[:w].hex(),
                  "dst": (b"\x08\xdc\xf0\x38" * 4)[:w].hex()})
    C.append({"fn": "inet", "data": hx(bytes.fromhex("010203040506")), "proto": 6,
              "src": ip("192.168.33.2").hex(), "dst": ip("192.168.33.1").hex()})
    # UDP datagrams of pip_udp.cpp:28-65 shape: 8-B header (uh_sum 0) + (i*13+1) payload
    for n, fam in ((8952, 6), (8951, 6), (1472, 4)):
        payload = pattern_bytes({"pattern": "affine", "len": n, "mul": 13, "add": 1})
        hdr = (5353).to_bytes(2, "big") + (53).to_bytes(2, "big") + (8 + n).to_bytes(2, "big") + b"\0\0"
        if fam == 6:
            C.append({"fn": "inet6_chain", "segs": [hx(hdr), {"pattern": "affine", "len": n, "mul": 13, "add": 1}],
                      "proto": 17, "src": v6(1).hex(), "dst": v6(2).hex()})
        else:
            C.append({"fn": "inet_chain", "segs": [hx(hdr), {"pattern": "affine", "len": n, "mul": 13, "add": 1}],
                      "proto": 17, "src": ip("10.0.0.1").hex(), "dst": ip("10.0.0.2").hex()})
        del payload
    # all-0xFF / all-zero around the 0x0000 vs 0xFFFF edge
    for fam in (4, 6):
        for byte in (0, 255):
            for n in (0, 1, 2, 7, 64, 1480, 8960):
                a = bytes([byte]) * (4 if fam == 4 else 16)
                C.append({"fn": "inet" if fam == 4 else "inet6", "data": {"pattern": "const", "byte": byte, "len": n},
                          "proto": 255 if byte else 0, "src": a.hex(), "dst": a.hex()})
    # random cases: every function, odd/even lengths, random initial sums, odd chains
    for _ in range(160):
        n = rng.choice([rng.randint(0, 64), rng.randint(0, 2000), rng.randint(8000, 9100)])
        data = {"pattern": "affine", "len": n, "mul": rng.randint(1, 255), "add": rng.randint(0, 255)}
        kind = rng.choice(["standard", "ip", "inet", "inet6", "inet_chain", "inet6_chain"])
        if kind == "standard":
            C.append({"fn": kind, "data": data, "sum": rng.choice([0, rng.getrandbits(16), rng.getrandbits(32)])})
        elif kind == "ip":
            C.append({"fn": kind, "data": data})
        elif kind in ("inet", "inet6"):
            w = 4 if kind == "inet" else 16
            C.append({"fn": kind, "data": data, "proto": rng.randint(0, 255),
                      "src": rng.randbytes(w).hex(), "dst": rng.randbytes(w).hex()})
        else:
            w = 4 if kind == "inet_chain" else 16
            segs = [{"pattern": "affine", "len": rng.choice([rng.randint(0, 7), rng.randint(1, 300), 20, 8]),
                     "mul": rng.randint(1, 255), "add": rng.randint(0, 255)} for _ in range(rng.randint(1, 5))]
            C.append({"fn": kind, "segs": segs, "proto": rng.randint(0, 255),
                      "src": rng.randbytes(w).hex(), "dst": rng.randbytes(w).hex()})
    # chains whose pip_buf::total_len passes 65,535 (missing 2): pip adds
    # the u32 total_len to the pseudo-header as hi + lo (pip_checksum.cpp:105-107,
    # 139-141), so the hi term is non-zero here; every segment stays <= 65,535 B
    for fam_fn, w in (("inet_chain", 4), ("inet6_chain", 16)):
        for lens in ([40000, 40000], [30001, 30001, 30001], [65535, 1], [65535] * 4):
            segs = [{"pattern": "affine", "len": L, "mul": rng.randint(1, 255), "add": rng.randint(0, 255)}
                    for L in lens]
            C.append({"fn": fam_fn, "segs": segs, "proto": rng.choice([6, 17]),
                      "src": rng.randbytes(w).hex(), "dst": rng.randbytes(w).hex()})
        # the largest sums pip's per-segment loop can carry: all-0xFF segments and addresses
        C.append({"fn": fam_fn, "segs": [{"pattern": "const", "byte": 255, "len": 65535}] * 4, "proto": 255,
                  "src": (b"\xff" * w).hex(), "dst": (b"\xff" * w).hex()})
    return C


def run_case(impl, c: dict) -> int:
    fn = c["fn"]
    if fn == "standard":
        return impl.standard_checksum(pattern_bytes(c["data"]), None, c["sum"])
    if fn == "ip":
        return impl.ip_checksum(pattern_bytes(c["data"]))
    if fn == "fold":
        return impl.fold_uint32(c["x"])
    s, d = bytes.fromhex(c["src"]), bytes.fromhex(c["dst"])
    if fn == "inet":
        return impl.inet_checksum(pattern_bytes(c["data"]), c["proto"], s, d)
    if fn == "inet6":
        return impl.inet6_checksum(pattern_bytes(c["data"]), c["proto"], s, d)
    segs = [pattern_bytes(x) for x in c["segs"]]
    if fn == "inet_chain":
        return impl.inet_checksum_chain(segs, c["proto"], s, d)
    if fn == "inet6_chain":
        return impl.inet6_checksum_chain(segs, c["proto"], s, d)
    raise ValueError(fn)


# reduced batch sizes per config (full sizes are for the GPU properties tests and the bench)
GOLDEN_N = {"cfg1_ipv4_header": 65536, "cfg2_tcp4_mtu1500": 16384, "cfg3_udp6_mtu9000": 2048,
            "cfg4_tcp4_zipf": 16384, "cfg5_tcp4_mtu9000": 2048}
GOLDEN_FIRST = {"cfg5_tcp4_mtu9000": 8 << 20}  # cfg5 shard of rank 1 of 8: ids start at 8M


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# Edge batches: a config's generated batch with some packets made to hit pip's
# fold corners.  "ck_every"/"ck_off": packet i (i % ck_every == 0) gets pip's
# own checksum of the unpatched packet stored big-endian at ck_off (its
# th_sum / uh_sum / ip_sum, zero in the generated bytes) -> that packet now
# checksums to 0x0000.  "zero_every": packet i (i % zero_every == 1) becomes all
# zero bytes -> 0xFFFF where there is no pseudo-header (pip_ip_checksum of an
# all-zero header).  "zero_flows_every": flow records k % zero_flows_every == 0
# get zero addresses; with proto 0 and length 0 (an empty segment) their total
# is 0 and pip returns 0xFFFF under a pseudo-header.  "family": 0 drops the
# config's pseudo-header (pip_ip_checksum semantics over the whole segment), so
# all-zero packets fold to pip's ~fold(0) = 0xFFFF (pip/pip_checksum.cpp:29-38)
# through the jumbo and byte-packed bench kernels too.  Each spec names the batch
# kernel it exercises (tests/test_gpu_parity.py checks pipck_last_launch), and
# fixed strides of 1 KiB and more also the other schedule ("alt", tune bit 28:
# k_flat where k_flat_coop is the default, and the reverse) on the same bytes.
EDGES = {
    "edge_flat24_tcp4": {"cfg": 2, "n": 192, "ck_every": 3, "ck_off": 16, "kernel": "k_flat_coop<32,",
                         "alt": "k_flat<24,"},
    "edge_flat32_udp6": {"cfg": 3, "n": 48, "ck_every": 2, "ck_off": 6, "kernel": "k_flat_coop<32,",
                         "alt": "k_flat<32,"},
    "edge_small_ip20": {"cfg": 1, "n": 4096, "ck_every": 5, "ck_off": 10, "zero_every": 7, "kernel": "k_small<"},
    "edge_packed_tcp4": {"cfg": 4, "n": 4096, "ck_every": 2, "ck_off": 16, "zero_every": 0, "kernel": "k_packed<"},
    "edge_packedb_tcp4": {"cfg": 4, "n": 4096, "ck_every": 3, "ck_off": 16, "zero_every": 0, "layout": "bytes",
                          "kernel": "k_packedb<"},
    "edge_flat_len0_v4": {"cfg": 2, "n": 256, "stride": 1024, "length": 0, "proto": 0, "zero_flows_every": 4,
                          "kernel": "k_flat<24,", "alt": "k_flat_coop<32,"},
    # no pseudo-header, all-zero packets -> 0xFFFF, self-checksummed ones -> 0x0000
    "edge_coop_nopseudo_tcp4": {"cfg": 5, "n": 96, "family": 0, "proto": 0, "ck_every": 4, "ck_off": 16,
                                "zero_every": 3, "kernel": "k_flat_coop<32,", "alt": "k_flat<32,"},
    "edge_packedb_nopseudo": {"cfg": 4, "n": 2048, "family": 0, "proto": 0, "ck_every": 5, "ck_off": 16,
                              "zero_every": 3, "layout": "bytes", "kernel": "k_packedb<"},
}


def edge_inputs_cpu(orc, b: dict):
    """Rebuild an edge fixture's inputs on the CPU from its record (generator twin +
    the recorded patches / zeroed flows): (arena, offsets, lengths, flow table bytes)."""
    w = next(x for x in ALL.values() if x.cfg == b["cfg"])
    n, fam = b["n"], b["family"]
    flows = bytearray(orc.flows_table(fam, b["seed"], b["n_flows"], b["proto"]) if fam else b"")
    rec = 12 if fam == 4 else 36
    for k in b["zero_flows"]:
        flows[rec * k:rec * k + rec - 4] = bytes(rec - 4)
    if w.ragged and b.get("layout") == "bytes":
        arena, offs, lens = orc.gen_packed_bytes_batch(b["seed"], b["first"], n, b["hdr"])
    elif w.ragged:
        arena, offs, lens = orc.gen_ragged_batch(b["seed"], b["first"], n, b["hdr"])
    else:
        st, L = b["stride"], b["length"]
        arena = orc.gen_fixed_batch(b["seed"], b["first"], n, L, b["hdr"], st) if L else np.zeros(n * st, np.uint8)
        offs, lens = np.arange(n, dtype=np.uint64) * st, np.full(n, L, dtype=np.uint32)
    for o, hx in b["patches"]:
        v = patch_bytes(hx)
        arena[o:o + len(v)] = np.frombuffer(v, dtype=np.uint8)
    return arena, offs, lens, bytes(flows)


def patch_bytes(p) -> bytes:
    """A fixture patch's bytes: hex text, or an int = that many zero bytes."""
    return bytes(p) if isinstance(p, int) else bytes.fromhex(p)


def oracle_edge_results(orc, b: dict, arena, offs, lens, flows: bytes) -> np.ndarray:
    """The oracle restatement, packet by packet, over an edge batch (its flow table may differ
    from the generator's, so the batch helpers that derive flows from the seed do not apply)."""
    fam, rec = b["family"], (12 if b["family"] == 4 else 36)
    out = np.zeros(b["n"], dtype=np.uint16)
    for i in range(b["n"]):
        o, L = int(offs[i]), int(lens[i])
        data = arena[o:o + L].tobytes()
        if not fam:
            out[i] = orc.ip_checksum(data)
        else:
            r = flows[rec * ((b["first"] + i) % b["n_flows"]):][:rec - 4]
            half = (rec - 4) // 2
            out[i] = (orc.inet_checksum if fam == 4 else orc.inet6_checksum)(data, b["proto"], r[:half], r[half:], L)
    return out


def edge_batch(orc, ref, name: str, spec: dict) -> dict:
    """Build one edge batch with pip's own code; return its fixture record."""
    w = next(x for x in ALL.values() if x.cfg == spec["cfg"])
    n, first = spec["n"], 0
    proto = spec.get("proto", w.proto)
    fam = spec.get("family", w.family)
    flows = bytearray(orc.flows_table(fam, w.seed, N_FLOWS, proto) if fam else b"")
    rec = 12 if fam == 4 else 36
    zero_flows = list(range(0, N_FLOWS, spec["zero_flows_every"])) if spec.get("zero_flows_every") else []
    for k in zero_flows:
        flows[rec * k:rec * k + rec - 4] = bytes(rec - 4)  # src, dst (proto stays)
    flows = bytes(flows)
    if w.ragged and spec.get("layout") == "bytes":
        arena, offs, lens = orc.gen_packed_bytes_batch(w.seed, first, n, w.hdr)
        stride, length = 0, None
    elif w.ragged:
        arena, offs, lens = orc.gen_ragged_batch(w.seed, first, n, w.hdr)
        stride, length = 0, None
    else:
        stride, length = spec.get("stride", w.stride), spec.get("length", w.length)
        arena = orc.gen_fixed_batch(w.seed, first, n, length, w.hdr, stride) if length else \
            np.zeros(n * stride, dtype=np.uint8)
        offs = np.arange(n, dtype=np.uint64) * stride
        lens = np.full(n, length, dtype=np.uint32)

    def pip_results(a):
        if w.ragged:
            return ref.batch_ragged(a, offs, lens, fam, proto, flows, N_FLOWS, first)
        return ref.batch_fixed(a, stride, length, n, fam, proto, flows, N_FLOWS, first)

    base = pip_results(arena)
    patches = []
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        if spec.get("zero_every") and i % spec["zero_every"] == 1:
            patches.append([o, L])  # an int: a run of L zero bytes
        elif spec.get("ck_every") and i % spec["ck_every"] == 0 and L >= spec["ck_off"] + 2:
            patches.append([o + spec["ck_off"], int(base[i]).to_bytes(2, "big").hex()])
    for o, hx in patches:
        b = patch_bytes(hx)
        arena[o:o + len(b)] = np.frombuffer(b, dtype=np.uint8)
    out = pip_results(arena)
    rec_ = {"n": n, "first": first, "family": fam, "proto": proto, "n_flows": N_FLOWS}
    assert np.array_equal(oracle_edge_results(orc, rec_, arena, offs, lens, flows), out), name
    n_zero, n_ffff = int((out == 0).sum()), int((out == 0xFFFF).sum())
    assert n_zero + n_ffff > 0, name
    return {"cfg": w.cfg, "n": n, "first": first, "seed": w.seed, "stride": stride, "length": length, "hdr": w.hdr,
            "family": fam, "proto": proto, "n_flows": N_FLOWS, "zero_flows": zero_flows, "patches": patches,
            "kernel": spec["kernel"], "alt": spec.get("alt"),
            "layout": spec.get("layout", "padded16" if w.ragged else "fixed"),
            "arena_sha256": sha(arena), "results_sha256": sha(out.astype("<u2")),
            "head": [int(x) for x in out[:16]], "n_zero": n_zero, "n_ffff": n_ffff}


def main() -> None:
    ref, orc = Reference(), Oracle()
    rng = random.Random(20261015)
    cases = kat_cases(rng)
    cases.extend({"fn": "fold", "x": x} for x in (0, 1, 0xFFFF, 0x10000, 0x1FFFE, 0xFFFFFFFF, 0x12345678))
    for c in cases:
        c["expect"] = run_case(ref, c)
        got = run_case(orc, c)
        assert got == c["expect"], (c, got)
    (OUT / "kat.json").write_text(json.dumps({"source": "pip/pip_checksum.cpp compiled from /root/reference",
                                              "cases": cases}, indent=0))
    print(f"kat.json: {len(cases)} cases")

    batches = {}
    for name, w in ALL.items():
        n, first = GOLDEN_N[name], GOLDEN_FIRST.get(name, 0)
        flows = orc.flows_table(w.family, w.seed, N_FLOWS, w.proto) if w.family else b""
        if w.ragged:
            arena, offs, lens = orc.gen_ragged_batch(w.seed, first, n, w.hdr)
            want = orc.batch_ragged(arena, offs, lens, w.family, w.proto, w.seed, N_FLOWS, first)
            # pip itself, packet by packet
            ref_out = np.array([ref.inet_checksum(arena[int(o):int(o) + int(L)].tobytes(), w.proto,
                                                  *orc.flow4(w.seed, (first + i) % N_FLOWS), int(L))
                                for i, (o, L) in enumerate(zip(offs, lens))], dtype=np.uint16)
            # the byte-packed layout the bench runs (pipck_checksum_packed_bytes): same packets, no padding
            ab, _, _ = orc.gen_packed_bytes_batch(w.seed, first, n, w.hdr)
            extra = {"lengths_sha256": sha(lens.astype("<u4")), "mean_len": float(lens.mean()),
                     "arena_bytes": int(arena.size), "arena_bytes_sha256": sha(ab)}
        else:
            arena = orc.gen_fixed_batch(w.seed, first, n, w.length, w.hdr, w.stride)
            want = orc.batch_fixed(arena, w.stride, w.length, n, w.family, w.proto, w.seed, N_FLOWS, first)
            ref_out = ref.batch_fixed(arena, w.stride, w.length, n, w.family, w.proto, flows, N_FLOWS, first)
            extra = {}
        assert np.array_equal(want, ref_out), name
        batches[name] = {"cfg": w.cfg, "n": n, "first": first, "seed": w.seed, "stride": w.stride,
                         "length": w.length, "hdr": w.hdr, "family": w.family, "proto": w.proto,
                         "n_flows": N_FLOWS, "arena_sha256": sha(arena), "results_sha256": sha(ref_out.astype("<u2")),
                         "head": [int(x) for x in ref_out[:16]], "n_zero": int((ref_out == 0).sum()),
                         "n_ffff": int((ref_out == 0xFFFF).sum()), **extra}
        print(name, n, batches[name]["results_sha256"][:16])
    for name, spec in EDGES.items():
        batches[name] = edge_batch(orc, ref, name, spec)
        print(name, batches[name]["n"], "zero", batches[name]["n_zero"], "ffff", batches[name]["n_ffff"])
    (OUT / "batches.json").write_text(json.dumps(batches, indent=1))

    out = subprocess.run([str(ROOT / "oracle" / "_ref" / "stack_replay_ref")], check=True, capture_output=True,
                         text=True).stdout
    assert out.strip().endswith("VERIFY_BAD 0"), out[-200:]
    (OUT / "stack_replay.txt").write_text(out)
    print("stack_replay.txt:", out.strip().splitlines()[-1])


if __name__ == "__main__":
    main()
