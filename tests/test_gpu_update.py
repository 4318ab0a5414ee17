"""GPU parity of the incremental update (RFC 1624).

The oracle for pipck_update_fixed is pip's own full recomputation: after the
rewrite, zero the checksum field and re-run pip's checksum (the oracle's
restatement of pip/pip_checksum.cpp:35-87) over the covered bytes; the patched
field must equal htons() of that result bit for bit, including the
0x0000 / 0xFFFF corner that RFC 1624 eqn. 3 alone cannot decide.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG1, CFG2, CFG3, N_FLOWS  # noqa: E402

DEV = "cuda"
FIELD = {CFG1.name: 10, CFG2.name: 16, CFG3.name: 6}  # ip_sum / th_sum / uh_sum


@pytest.fixture(scope="module", autouse=True)
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a visible MI355X"
    engine.require_gpu()
    yield
    torch.cuda.synchronize()


def _store_be(arena, stride, n, field, out):
    rows = arena.view(n, stride)
    v = out.to(torch.int32) & 0xFFFF
    rows[:, field] = (v >> 8).to(torch.uint8)
    rows[:, field + 1] = (v & 0xFF).to(torch.uint8)


def _field(host: np.ndarray, stride, n, field) -> np.ndarray:
    rows = host.reshape(n, stride)
    return (rows[:, field].astype(np.uint16) << 8) | rows[:, field + 1]


def _recompute(oracle, host, w, n, field, family, seed):
    """pip's full recomputation of the edited batch (field zeroed first)."""
    z = host.copy().reshape(n, w.stride)
    z[:, field:field + 2] = 0
    return oracle.batch_fixed(z.reshape(-1), w.stride, w.length, n, family, w.proto, seed, N_FLOWS, threads=8)


@pytest.mark.parametrize("w,edit_off,edit_len,nat", [
    (CFG1, 12, 8, False),   # IPv4 header: rewrite src + dst (ip_sum, pip_netif.cpp:94-97)
    (CFG1, 8, 2, False),    # TTL / proto word
    (CFG2, 4, 8, False),    # TCP seq + ack
    (CFG2, 0, 4, True),     # TCP ports + NAT of the v4 addresses (pseudo-header change)
    (CFG3, 0, 4, True),     # UDP/IPv6 ports + v6 address rewrite
    (CFG2, 0, 0, True),     # pseudo-header change only
])
def test_update_matches_pip_recompute(oracle, w, edit_off, edit_len, nat):
    n = 30000 if w.length > 1000 else 200000
    field = FIELD[w.name]
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device=DEV)
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    p_old = p_new = None
    seed_new = w.seed
    if w.family:
        _, p_old = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)
        if nat:
            seed_new = w.seed ^ 0x5EED
            _, p_new = engine.gen_flows(w.family, N_FLOWS, seed_new, w.proto)
        else:
            p_new = p_old
    out = engine.checksum_fixed(arena, w.stride, w.length, n, p_old, N_FLOWS)
    _store_be(arena, w.stride, n, field, out)
    g = torch.Generator(device="cpu").manual_seed(7 + edit_off)
    new = torch.randint(0, 256, (n, 8), dtype=torch.uint8, generator=g)
    new[::97] = 0          # all-zero edits
    new[1::97] = 0xFF      # all-0xFF edits
    new_d = new.to(DEV)
    engine.update_fixed(arena, w.stride, n, 0, w.length, field, edit_off, edit_len, new_d.view(-1), 8,
                        p_old, p_new, N_FLOWS)
    host = arena.cpu().numpy()
    rows = host.reshape(n, w.stride)
    assert np.array_equal(rows[:, edit_off:edit_off + edit_len], new.numpy()[:, :edit_len])
    want = _recompute(oracle, host, w, n, field, w.family, seed_new)
    got = _field(host, w.stride, n, field)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: got {got[bad[:5]]} want {want[bad[:5]]}"
    ok = engine.verify_fixed(arena, w.stride, w.length, n, p_new, N_FLOWS)
    assert bool((ok == 1).all())


def _corner_batch(rng, n, cover):
    """Packets of bytes drawn from {0x00, 0xFF} (mostly zero) so that sums of
    0 and of multiples of 0xFFFF -- the 0x0000 / 0xFFFF corner -- are common."""
    sparse = rng.random((n, cover)) < 0.08
    return np.where(sparse, 0xFF, 0).astype(np.uint8)


@pytest.mark.parametrize("cover,ck_off,edit_off,edit_len", [
    (8, 0, 2, 2), (8, 6, 0, 6), (9, 0, 2, 7), (20, 10, 12, 8), (3, 0, 2, 1),
])
def test_update_corner_cases_ip(oracle, cover, ck_off, edit_off, edit_len):
    rng = np.random.default_rng(cover * 131 + edit_off)
    n = 20000
    stride = cover + 1
    pk = np.zeros((n, stride), dtype=np.uint8)
    pk[:, :cover] = _corner_batch(rng, n, cover)
    pk[:, ck_off:ck_off + 2] = 0
    pk[: n // 4, :cover] = 0  # all-zero packets: pip stores 0xFFFF
    pk[: n // 4, ck_off:ck_off + 2] = 0
    for i in range(n):
        c = oracle.ip_checksum(pk[i, :cover].tobytes())
        pk[i, ck_off], pk[i, ck_off + 1] = c >> 8, c & 0xFF
    new = np.where(rng.random((n, 8)) < 0.3, 0xFF, 0).astype(np.uint8)
    arena = torch.from_numpy(pk.reshape(-1).copy()).to(DEV)
    engine.update_fixed(arena, stride, n, 0, cover, ck_off, edit_off, edit_len, torch.from_numpy(new).to(DEV).view(-1),
                        8)
    got = arena.cpu().numpy().reshape(n, stride)
    exp = pk.copy()
    exp[:, edit_off:edit_off + edit_len] = new[:, :edit_len]
    exp[:, ck_off:ck_off + 2] = 0
    for i in range(n):
        c = oracle.ip_checksum(exp[i, :cover].tobytes())
        exp[i, ck_off], exp[i, ck_off + 1] = c >> 8, c & 0xFF
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first rows {bad[:5]}"
    # the corner must actually have been exercised both ways
    ck = (exp[:, ck_off].astype(np.uint16) << 8) | exp[:, ck_off + 1]
    assert (ck == 0xFFFF).any()
    if cover >= 8:
        assert (ck == 0).any()


def test_update_corner_cases_pseudo(oracle):
    """Zero pseudo-headers (0.0.0.0 -> 0.0.0.0, proto 0) next to real ones."""
    rng = np.random.default_rng(5)
    n, cover, stride, ck_off = 8000, 6, 8, 4
    flows = bytearray()
    addrs = []
    for f in range(4):
        s = bytes(4) if f < 2 else bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        d = bytes(4) if f < 2 else bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        proto = 0 if f == 0 else 6
        flows += s + d + bytes([proto, 0, 0, 0])
        addrs.append((s, d, proto))
    fl = engine.flows_to_device(4, bytes(flows))
    pseudo = engine.prepare_flows(4, fl, 4)
    pk = np.zeros((n, stride), dtype=np.uint8)
    pk[:, :cover] = _corner_batch(rng, n, cover)
    pk[:, ck_off:ck_off + 2] = 0

    def pip(row, f):
        s, d, proto = addrs[f]
        return oracle.inet_checksum(row[:cover].tobytes(), proto, s, d)

    for i in range(n):
        c = pip(pk[i], i % 4)
        pk[i, ck_off], pk[i, ck_off + 1] = c >> 8, c & 0xFF
    new = np.where(rng.random((n, 8)) < 0.3, 0xFF, 0).astype(np.uint8)
    arena = torch.from_numpy(pk.reshape(-1).copy()).to(DEV)
    engine.update_fixed(arena, stride, n, 0, cover, ck_off, 0, 4, torch.from_numpy(new).to(DEV).view(-1), 8,
                        pseudo, pseudo, 4)
    got = arena.cpu().numpy().reshape(n, stride)
    exp = pk.copy()
    exp[:, 0:4] = new[:, :4]
    exp[:, ck_off:ck_off + 2] = 0
    for i in range(n):
        c = pip(exp[i], i % 4)
        exp[i, ck_off], exp[i, ck_off + 1] = c >> 8, c & 0xFF
    bad = np.nonzero((got != exp).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first rows {bad[:5]}"
